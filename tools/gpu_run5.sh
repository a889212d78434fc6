#!/bin/bash
# GPU pass 5: tests, headline bench (MIOpen find on), BASELINE configs.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > gpurun_out/bench5.log 2>&1; rc=$?
tail -3 gpurun_out/bench5.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --batch 512 --no-baseline > gpurun_out/bench5_b512.log 2>&1; rc=$?
tail -1 gpurun_out/bench5_b512.log
[ $rc -eq 0 ] || exit $rc
for c in resnet_trimmed resnet_mkrum bert_geomed; do
  timeout -k 10 600 python bench/configs.py --config $c --steps 10 --warmup 3 --virtual-workers 8 --batch 32 --json-out gpurun_out/configs5.jsonl > gpurun_out/cfg5_$c.log 2>&1; rc=$?
  tail -1 gpurun_out/cfg5_$c.log
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 900 python bench/configs.py --config llama_gossip --steps 5 --warmup 2 --json-out gpurun_out/configs5.jsonl > gpurun_out/cfg5_llama.log 2>&1; rc=$?
tail -2 gpurun_out/cfg5_llama.log
exit $rc
