#!/bin/bash
# Round 4, GPU pass 37: batch-256 step, own 1x1 weight gradients for all nine >= 128-channel shapes
# (CML_WGRAD1X1_SET=all) vs the batch-2048-tuned five (core), three alternating pairs on one box;
# then a kernel profile of the "all" step (which library kernels remain at batch 256).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_37; mkdir -p $O
cd $R
for i in 1 2 3; do
  for s in core all; do
    CML_WGRAD1X1_SET=$s timeout -k 10 200 python -u bench.py --batch 256 --steps 40 --warmup 8 --no-baseline --b256-batch 0 --virtual-workers 0 --json-out $O/b256_${s}_$i.json > $O/b256_${s}_$i.log 2>&1 || { tail -20 $O/b256_${s}_$i.log; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'])" $O/b256_${s}_$i.json $s
  done
done
cd /tmp && export TMPDIR=/tmp
CML_WGRAD1X1_SET=all timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw -o run -- python3 $R/bench.py --batch 256 --steps 10 --warmup 5 --no-baseline --b256-batch 0 --virtual-workers 0 --profile-marker > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
db=$(find $O/raw -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 10 --top 400 --out $O/kernels_b256_all.md
python3 $R/tools/kernel_classes.py $O/kernels_b256_all.md > $O/classes_b256_all.md || true
rm -rf $O/raw
sed -n 1,3p $O/kernels_b256_all.md
cat $O/classes_b256_all.md
