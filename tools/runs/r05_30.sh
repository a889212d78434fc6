#!/bin/bash
# r05 pass 30: re-tune the ResNet fusion knobs after the weight-gradient changes (alternating
# with the defaults, 30 timed steps each).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_30; mkdir -p $O
cd $R
run() {   # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-baseline --b256-batch 0 --virtual-workers 0 > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  echo "$tag $(grep '^{' $O/$tag.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
}
for rep in 1 2; do
run base_$rep CML_NONE=1
run rt128_$rep CML_RECOMPUTE_TAIL_MAX_PLANES=128
run rt512_$rep CML_RECOMPUTE_TAIL_MAX_PLANES=512
run fb256_$rep CML_FUSED_BN3_BWD_MAX_PLANES=256
run gemm_$rep CML_CONV1X1_GEMM=gemm
run ds1024_$rep CML_DOWN_TAIL_S2_MAX_CIN=1024
run cat128_$rep CML_CAT_BNSUMS_MAXC=128
done
