#!/bin/bash
# r06 pass 37: 4 gloo ranks sharing cuda:0 stopped after the warmup step in pass 36: the same run
# with periodic Python stack dumps to see where each rank waits.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_37; mkdir -p $O
cd $R
CML_TRACEBACK_AFTER=45 timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29614 bench.py --gpus 4 --dist-backend gloo --batch 128 --steps 3 --warmup 1 --b256-batch 0 --virtual-workers 0 --no-baseline > $O/gloo4.log 2>&1
echo "rc=$?"
grep -c "Thread\|File" $O/gloo4.log
