#!/bin/bash
# Round 2, GPU pass 14: A/B of the fused identity-tail backward (CML_FUSED_BN3_BWD) + kernel
# profile of the fused step.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -f $O/r02_14_*
for f in 0 1; do
CML_FUSED_BN3_BWD=$f timeout -k 10 400 python -u bench.py --steps 15 --warmup 5 --no-baseline --virtual-workers 0 > $O/r02_14_bench$f.log 2>&1 || { tail -20 $O/r02_14_bench$f.log; exit 1; }
echo "fused_bn3_bwd=$f $(grep -o '"ms_per_step": [0-9.]*' $O/r02_14_bench$f.log)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw14 -o run -- python3 $R/bench.py --steps 6 --warmup 2 --no-baseline --virtual-workers 0 --profile-marker > $O/r02_14_prof.log 2>&1 || { tail -20 $O/r02_14_prof.log; exit 1; }
db=$(find $O/raw14 -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 70 --out $O/r02_14_kernels.md
rm -rf $O/raw14
head -45 $O/r02_14_kernels.md | cut -c1-200
