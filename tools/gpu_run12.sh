#!/bin/bash
# GPU pass 12 (fresh container rebuild check): GPU tests, headline bench, and kernel profiles of
# the transformer configs (BERT-base geomed, Llama-3-8B gossip) to find their hot kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu12.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu12.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --json-out gpurun_out/bench12.json > gpurun_out/bench12.log 2>&1; rc=$?
tail -1 gpurun_out/bench12.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof12_bert -o run -- python3 $R/bench/configs.py --config bert_geomed --virtual-workers 8 --batch 32 --steps 4 --warmup 2 > $R/gpurun_out/prof12_bert.log 2>&1; rc=$?
tail -1 $R/gpurun_out/prof12_bert.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof12_llama -o run -- python3 $R/bench/configs.py --config llama_gossip --steps 3 --warmup 2 > $R/gpurun_out/prof12_llama.log 2>&1; rc=$?
tail -1 $R/gpurun_out/prof12_llama.log | cut -c1-300
exit $rc
