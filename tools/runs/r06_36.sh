#!/bin/bash
# r06 pass 36: multi-rank rehearsal of the bench on one GPU (gloo, 2 and 4 ranks sharing cuda:0):
# the sharded Krum exchange, the selection and the replica check at N > 1 on the final code.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_36; mkdir -p $O
cd $R
for n in 2 4; do
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2961$n bench.py --gpus $n --dist-backend gloo --batch 128 --steps 3 --warmup 1 --b256-batch 0 --virtual-workers 0 --no-baseline > $O/gloo$n.log 2>&1 || { tail -30 $O/gloo$n.log; exit 1; }
  grep '^{' $O/gloo$n.log > $O/gloo$n.json
  python3 -c "
import json
r=json.loads(open('$O/gloo$n.json').readline())
print('gloo $n', {k: r.get(k) for k in ['value','n_gpus','world_size_seen','replicas_identical','loss_finite','selection','dist_backend']})"
done
