#!/bin/bash
# Round 2, GPU pass 29: full GPU suite, default bench (Krum + virtual Krum block), steady-state
# kernel profile of the current default step.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r02_29_* $O/raw29
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r02_29_pytest.log 2>&1 || { tail -40 $O/r02_29_pytest.log; exit 1; }
tail -1 $O/r02_29_pytest.log
timeout -k 10 600 python -u bench.py > $O/r02_29_bench.log 2>&1 || { tail -20 $O/r02_29_bench.log; exit 1; }
grep '"metric"' $O/r02_29_bench.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw29 -o run -- python3 $R/bench.py --steps 6 --warmup 2 --no-baseline --virtual-workers 0 --profile-marker > $O/r02_29_prof.log 2>&1 || { tail -20 $O/r02_29_prof.log; exit 1; }
db=$(find $O/raw29 -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 90 --out $O/r02_29_kernels.md
rm -rf $O/raw29
python3 $R/tools/kernel_classes.py $O/r02_29_kernels.md
