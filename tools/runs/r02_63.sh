#!/bin/bash
# Round 2, GPU pass 63: one-launch BN affine (bn_affine) in the fused conv paths: numerics (bit
# identity + fusion tests), step A/B against the PyTorch ops (CML_BN_AFFINE_KERNEL=0).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r02_63_*
timeout -k 10 400 python -u -m pytest tests/test_bwd_fusion_gpu.py tests/test_conv1x1_bn_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/r02_63_pytest.log 2>&1 || { tail -40 $O/r02_63_pytest.log; exit 1; }
tail -1 $O/r02_63_pytest.log
for a in 1 0 1 0; do
CML_BN_AFFINE_KERNEL=$a timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-baseline --virtual-workers 0 > $O/r02_63_bench_$a.log 2>&1 || { tail -20 $O/r02_63_bench_$a.log; exit 1; }
echo "bn_affine_kernel=$a $(grep -o '"ms_per_step": [0-9.]*' $O/r02_63_bench_$a.log)"
done
