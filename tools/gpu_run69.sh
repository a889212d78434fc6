#!/bin/bash
# GPU pass 69: per-GPU batch 1536 vs 2048.
set -o pipefail
cd $GRAFT_REPO_ROOT
for b in 1536 2048 1536 2048; do
  timeout -k 10 400 python bench.py --batch $b --steps 20 --warmup 3 --no-baseline --json-out gpurun_out/bench69_b$b.json > gpurun_out/bench69_b$b.log 2>&1 || exit $?
  echo "b$b $(tail -1 gpurun_out/bench69_b$b.log | cut -c90-190)"
done
python - <<'PY'
import torch
print("device mem GB", torch.cuda.get_device_properties(0).total_memory / 2**30)
PY
