#!/bin/bash
# Round 2, GPU pass 8: full GPU suite (new multi-rank gossip / robust-rule / prefetch tests),
# then a 2-rank gloo rehearsal of bench.py's N > 1 path (ranks share cuda:0).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r02_08_pytest.log 2>&1 || { tail -40 $O/r02_08_pytest.log; exit 1; }
tail -2 $O/r02_08_pytest.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --dist-backend gloo --batch 256 --steps 3 --warmup 1 > $O/r02_08_gloo2.log 2>&1 || { tail -30 $O/r02_08_gloo2.log; exit 1; }
grep '"metric"' $O/r02_08_gloo2.log | cut -c1-2000
