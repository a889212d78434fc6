#!/bin/bash
# Round 2, GPU pass 60: policy re-check with the current kernels -- layer-4 identity tails on the
# recompute kernels (CML_RECOMPUTE_TAIL_MAX_PLANES=512), layer-4 tails with bn3's backward fused
# (CML_FUSED_BN3_BWD_MAX_PLANES=512), stride-2 3x3 forward on conv_gemm (CML_CONV3X3_S2=1).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r02_60_*
run() {
  env $2 timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-baseline --virtual-workers 0 > $O/r02_60_bench_$1.log 2>&1 || { tail -20 $O/r02_60_bench_$1.log; exit 1; }
  echo "$1 $(grep -o '"ms_per_step": [0-9.]*' $O/r02_60_bench_$1.log)"
}
for r in 1 2; do
run default CML_NONE=0
run rec512 CML_RECOMPUTE_TAIL_MAX_PLANES=512
run bn3bwd512 CML_FUSED_BN3_BWD_MAX_PLANES=512
run conv3x3s2 CML_CONV3X3_S2=1
done
