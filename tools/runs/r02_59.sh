#!/bin/bash
# Round 2, GPU pass 59: layer-4 stride-2 downsample tail on the recompute kernels
# (CML_DOWN_TAIL_S2_MAX_CIN=1024) -- numerics, then step A/B against 512 (layers 2-3).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r02_59_*
timeout -k 10 400 python -u -m pytest tests/test_bwd_fusion_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "downsample_recompute" > $O/r02_59_pytest.log 2>&1 || { tail -40 $O/r02_59_pytest.log; exit 1; }
tail -1 $O/r02_59_pytest.log
for c in 1024 512 1024 512; do
CML_DOWN_TAIL_S2_MAX_CIN=$c timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-baseline --virtual-workers 0 > $O/r02_59_bench_$c.log 2>&1 || { tail -20 $O/r02_59_bench_$c.log; exit 1; }
echo "down_tail_s2_max_cin=$c $(grep -o '"ms_per_step": [0-9.]*' $O/r02_59_bench_$c.log) $(grep -o '"peak_mem_gib": [0-9.]*' $O/r02_59_bench_$c.log)"
done
