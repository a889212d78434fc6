#!/bin/bash
# r06 pass 45: batch-2560 A/B of this session's launch folding (finalize affine / dgamma, batched
# weight layouts + transposes) on one box, alternating.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_45; mkdir -p $O
cd $R
for i in 1 2; do
  for f in 1 0; do
    CML_FIN_AFFINE=$f CML_FIN_DGAMMA=$f CML_BATCH_WLAYOUTS=$f timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 \
      --no-baseline --b256-batch 0 --virtual-workers 0 > $O/ab_${f}_$i.log 2>&1 || { tail -20 $O/ab_${f}_$i.log; exit 1; }
    echo "fin=$f run $i: $(grep '^{' $O/ab_${f}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
