#!/bin/bash
# Round 2, GPU pass 25: 3x3 data gradient on conv_gemm.hip -- numerics + bench A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -f $O/r02_25_*
timeout -k 10 400 python -u -m pytest tests/test_conv1x1_bn_gpu.py tests/test_bwd_fusion_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/r02_25_pytest.log 2>&1 || { tail -30 $O/r02_25_pytest.log; exit 1; }
tail -1 $O/r02_25_pytest.log
for f in 0 1; do
CML_DGRAD3X3=$f timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-baseline --virtual-workers 0 > $O/r02_25_bench$f.log 2>&1 || { tail -20 $O/r02_25_bench$f.log; exit 1; }
echo "dgrad3x3=$f $(grep -o '"ms_per_step": [0-9.]*' $O/r02_25_bench$f.log)"
done
