#!/bin/bash
# Round 2, GPU pass 47: bn_stats_gram with 16 channels per workgroup; conv1x1 MT = 2 tiles with
# resident W (CML_C1_MT2_WRES): numerics under both settings, bench A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r02_47_*
timeout -k 10 400 python -u -m pytest tests/test_bwd_fusion_gpu.py tests/test_conv1x1_bn_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/r02_47_pytest0.log 2>&1 || { tail -40 $O/r02_47_pytest0.log; exit 1; }
tail -1 $O/r02_47_pytest0.log
CML_C1_MT2_WRES=1 timeout -k 10 400 python -u -m pytest tests/test_bwd_fusion_gpu.py tests/test_conv1x1_bn_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/r02_47_pytest1.log 2>&1 || { tail -40 $O/r02_47_pytest1.log; exit 1; }
tail -1 $O/r02_47_pytest1.log
for f in 0 1 0 1; do
CML_C1_MT2_WRES=$f timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-baseline --virtual-workers 0 > $O/r02_47_bench$f.log 2>&1 || { tail -20 $O/r02_47_bench$f.log; exit 1; }
echo "mt2_wres=$f $(grep -o '"ms_per_step": [0-9.]*' $O/r02_47_bench$f.log)"
done
