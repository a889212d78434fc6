#!/bin/bash
# r06 pass 57: A/B of the two sweep candidates at batch 2560 (CML_WGRAD1X1_SET=all,
# CML_FOLD_WIDE_MIN=64), alternating with the default.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_57; mkdir -p $O
cd $R
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --steps 20 --warmup 4 --no-baseline --b256-batch 0 \
    --virtual-workers 0 > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  echo "$tag: $(grep '^{' $O/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
}
for i in 1 2 3; do
  run base_$i CML_NOP=1
  run wgall_$i CML_WGRAD1X1_SET=all
  run fold64_$i CML_FOLD_WIDE_MIN=64
done
