#!/bin/bash
# Round 4, GPU pass 34: XCD-contiguous band mapping of the stem's fused BN + ReLU + max-pool forward:
# the BN / stem GPU tests, then the batch-2048 kernel profile (the pool kernel's time vs pass 33).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_34; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_bn_gpu.py tests/test_stem_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/quick.txt 2>&1 || { tail -40 $O/quick.txt; exit 1; }
tail -1 $O/quick.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw -o run -- python3 $R/bench.py --steps 6 --warmup 3 --no-baseline --b256-batch 0 --virtual-workers 0 --profile-marker > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
db=$(find $O/raw -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 400 --out $O/kernels_b2048.md
python3 $R/tools/kernel_classes.py $O/kernels_b2048.md > $O/classes_b2048.md || true
rm -rf $O/raw
grep -n "maxpool_fwd_k3s2" $O/kernels_b2048.md | cut -c1-200
