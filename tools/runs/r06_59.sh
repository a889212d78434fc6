#!/bin/bash
# r06 pass 59: final same-box A/B of the side-stream 3x3 weight gradients at batch 2560 (default on
# vs CML_SIDE_WGRAD=0), alternating, on the final code.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_59; mkdir -p $O
cd $R
for i in 1 2 3 4; do
  for f in 1 0; do
    CML_SIDE_WGRAD=$f timeout -k 10 300 python3 bench.py --steps 20 --warmup 4 --no-baseline --b256-batch 0 \
      --virtual-workers 0 > $O/side_${f}_$i.log 2>&1 || { tail -20 $O/side_${f}_$i.log; exit 1; }
    echo "side=$f run $i: $(grep '^{' $O/side_${f}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
