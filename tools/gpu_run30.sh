#!/bin/bash
# GPU pass 30: ResNet-50 Krum per-GPU batch 256 / 768 / 1024 vs the 512 default.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for b in 1024 768 256; do
timeout -k 10 400 python bench.py --steps 12 --warmup 3 --batch $b --no-baseline --json-out gpurun_out/bench30_b$b.json > gpurun_out/bench30_b$b.log 2>&1 || exit $?
echo "b=$b $(tail -1 gpurun_out/bench30_b$b.log | cut -c90-200) $(grep 'warmup [0-9]' gpurun_out/bench30_b$b.log)"
done
