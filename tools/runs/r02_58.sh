#!/bin/bash
# Round 2, GPU pass 58: layer-3 stride-2 downsample tail on the recompute kernels
# (CML_DOWN_TAIL_S2_MAX_CIN=512) -- numerics, then step A/B against 256 (layer 2 only).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r02_58_*
timeout -k 10 400 python -u -m pytest tests/test_bwd_fusion_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "downsample_recompute" > $O/r02_58_pytest.log 2>&1 || { tail -40 $O/r02_58_pytest.log; exit 1; }
tail -1 $O/r02_58_pytest.log
for c in 512 256 512 256; do
CML_DOWN_TAIL_S2_MAX_CIN=$c timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-baseline --virtual-workers 0 > $O/r02_58_bench_$c.log 2>&1 || { tail -20 $O/r02_58_bench_$c.log; exit 1; }
echo "down_tail_s2_max_cin=$c $(grep -o '"ms_per_step": [0-9.]*' $O/r02_58_bench_$c.log) $(grep -o '"peak_mem_gib": [0-9.]*' $O/r02_58_bench_$c.log)"
done
