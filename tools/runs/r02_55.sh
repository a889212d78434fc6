#!/bin/bash
# Round 2, GPU pass 55: 2-rank gloo rehearsal of the bench's N > 1 path (both ranks on cuda:0)
# with the current kernels: self-validation fields (world_size_seen, replicas_identical).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r02_55_*
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --dist-backend gloo --batch 256 --steps 3 --warmup 1 > $O/r02_55_gloo2.log 2>&1 || { tail -30 $O/r02_55_gloo2.log; exit 1; }
grep '"metric"' $O/r02_55_gloo2.log > $O/r02_55_gloo2.json
cut -c1-3000 $O/r02_55_gloo2.json
