#!/bin/bash
# r06 pass 53: CML_SIDE_WGRAD (3x3 weight gradients on a side stream) at batch 2560 and 256,
# alternating on / off on one box.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_53; mkdir -p $O
cd $R
for i in 1 2 3; do
  for f in 1 0; do
    CML_SIDE_WGRAD=$f timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-baseline --b256-batch 0 \
      --virtual-workers 0 > $O/b2560_${f}_$i.log 2>&1 || { tail -20 $O/b2560_${f}_$i.log; exit 1; }
    echo "b2560 side=$f run $i: $(grep '^{' $O/b2560_${f}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
for i in 1 2; do
  for f in 1 0; do
    CML_SIDE_WGRAD=$f timeout -k 10 300 python3 bench.py --batch 256 --steps 40 --warmup 8 --no-baseline \
      --b256-batch 0 > $O/b256_${f}_$i.log 2>&1 || { tail -20 $O/b256_${f}_$i.log; exit 1; }
    echo "b256 side=$f run $i: $(grep '^{' $O/b256_${f}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
