#!/bin/bash
# Round 2, GPU pass 37 (fresh container re-entry): full GPU suite, default bench (driver contract), step profile.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r02_37_* $O/raw37
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r02_37_gputests.txt 2>&1 || { tail -40 $O/r02_37_gputests.txt; exit 1; }
tail -1 $O/r02_37_gputests.txt
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r02_37_smoke.log 2>&1 || { tail -20 $O/r02_37_smoke.log; exit 1; }
tail -1 $O/r02_37_smoke.log
timeout -k 10 500 python -u bench.py > $O/r02_37_bench.log 2>&1 || { tail -20 $O/r02_37_bench.log; exit 1; }
grep '^{' $O/r02_37_bench.log > $O/r02_37_bench.json
cut -c1-300 $O/r02_37_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw37 -o run -- python3 $R/bench.py --steps 6 --warmup 2 --no-baseline --virtual-workers 0 --profile-marker > $O/r02_37_prof.log 2>&1 || { tail -20 $O/r02_37_prof.log; exit 1; }
db=$(find $O/raw37 -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 90 --out $O/r02_37_kernels.md
rm -rf $O/raw37
python3 $R/tools/kernel_classes.py $O/r02_37_kernels.md
