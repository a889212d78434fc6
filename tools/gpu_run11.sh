#!/bin/bash
# GPU pass 11: profile the transformer configs (BERT-base geomed, Llama-tiny gossip) to find their
# hot kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof11_bert -o run -- python3 $GRAFT_REPO_ROOT/bench/configs.py --config bert_geomed --virtual-workers 8 --batch 64 --steps 4 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof11_bert.log 2>&1; rc=$?
tail -1 $GRAFT_REPO_ROOT/gpurun_out/prof11_bert.log | cut -c1-400
exit $rc
