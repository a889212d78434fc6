#!/bin/bash
# Round 2, GPU pass 40: 3x3 weight gradients on wgrad3x3.hip in the model -- full GPU suite, bench
# A/B (CML_WGRAD3X3), step profile.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r02_40_* $O/raw40
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r02_40_gputests.txt 2>&1 || { tail -40 $O/r02_40_gputests.txt; exit 1; }
tail -1 $O/r02_40_gputests.txt
for f in 0 1 0 1; do
CML_WGRAD3X3=$f timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-baseline --virtual-workers 0 > $O/r02_40_bench$f.log 2>&1 || { tail -20 $O/r02_40_bench$f.log; exit 1; }
echo "wgrad3x3=$f $(grep -o '"ms_per_step": [0-9.]*' $O/r02_40_bench$f.log)"
done
grep '^{' $O/r02_40_bench1.log > $O/r02_40_bench_on.json
grep '^{' $O/r02_40_bench0.log > $O/r02_40_bench_off.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw40 -o run -- python3 $R/bench.py --steps 6 --warmup 2 --no-baseline --virtual-workers 0 --profile-marker > $O/r02_40_prof.log 2>&1 || { tail -20 $O/r02_40_prof.log; exit 1; }
db=$(find $O/raw40 -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 90 --out $O/r02_40_kernels.md
rm -rf $O/raw40
python3 $R/tools/kernel_classes.py $O/r02_40_kernels.md
