#!/bin/bash
# r06 pass 52: re-check of older PerfPolicy switches at batch 2560 on the current kernels (one box,
# baseline between every variant).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_52; mkdir -p $O
cd $R
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --steps 15 --warmup 4 --no-baseline --b256-batch 0 \
    --virtual-workers 0 > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  echo "$tag: $(grep '^{' $O/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
}
run base1 CML_NOP=1
run side_wgrad CML_SIDE_WGRAD=1
run base2 CML_NOP=1
run bn1_lib CML_BN1_SUMS_LIB_CONV1=1
run base3 CML_NOP=1
run rec512 CML_RECOMPUTE_TAIL_MAX_PLANES=512
run base4 CML_NOP=1
run bn3bwd256 CML_FUSED_BN3_BWD_MAX_PLANES=256
run base5 CML_NOP=1
run catmax512 CML_CAT_BNSUMS_MAXC=512
run base6 CML_NOP=1
