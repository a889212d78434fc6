#!/bin/bash
# Round 2, GPU pass 53: kernel profile of the default step (wide fold, bn2 / bn1 backward sums from
# the data-gradient epilogues) and of CML_BN1_DGRAD_SUMS=0 for the per-kernel A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r02_53_* $O/raw53*
cd /tmp && export TMPDIR=/tmp
for b in 1 0; do
CML_BN1_DGRAD_SUMS=$b timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw53_$b -o run -- python3 $R/bench.py --steps 6 --warmup 2 --no-baseline --virtual-workers 0 --profile-marker > $O/r02_53_prof$b.log 2>&1 || { tail -20 $O/r02_53_prof$b.log; exit 1; }
db=$(find $O/raw53_$b -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 90 --out $O/r02_53_kernels_bn1_$b.md
rm -rf $O/raw53_$b
python3 $R/tools/kernel_classes.py $O/r02_53_kernels_bn1_$b.md
done
