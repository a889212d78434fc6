#!/bin/bash
# GPU pass 55: per-GPU batch 512 vs 1024 (find-db now holds both batch sizes).
set -o pipefail
cd $GRAFT_REPO_ROOT
for b in 512 1024 512 1024; do
  timeout -k 10 400 python bench.py --batch $b --steps 20 --warmup 3 --no-baseline --json-out gpurun_out/bench55_b$b.json > gpurun_out/bench55_b$b.log 2>&1 || exit $?
  echo "b$b $(tail -1 gpurun_out/bench55_b$b.log | cut -c90-190)"
done
