#!/bin/bash
# r06 pass 56: more kernel-variant switches re-checked at batch 2560 on the final code (one box,
# a baseline between every variant).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_56; mkdir -p $O
cd $R
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --steps 15 --warmup 4 --no-baseline --b256-batch 0 \
    --virtual-workers 0 > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  echo "$tag: $(grep '^{' $O/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
}
run base1 CML_NOP=1
run foldwide16 CML_FOLD_WIDE_MIN=16
run base2 CML_NOP=1
run foldwide64 CML_FOLD_WIDE_MIN=64
run base3 CML_NOP=1
run ns128_8 CML_WGRAD_DMA_NS128=8
run base4 CML_NOP=1
run c1g_regstage CML_C1G=0
run base5 CML_NOP=1
run wgset_all CML_WGRAD1X1_SET=all
run base6 CML_NOP=1
run gm8 CML_GEMM_GM=8
run base7 CML_NOP=1
