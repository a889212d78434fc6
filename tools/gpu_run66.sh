#!/bin/bash
# GPU pass 66: per-GPU batch 1024 vs 1536 (find-db now holds 512 / 1024 / 1536).
set -o pipefail
cd $GRAFT_REPO_ROOT
for b in 1024 1536 1024 1536; do
  timeout -k 10 400 python bench.py --batch $b --steps 20 --warmup 3 --no-baseline --json-out gpurun_out/bench66_b$b.json > gpurun_out/bench66_b$b.log 2>&1 || exit $?
  echo "b$b $(tail -1 gpurun_out/bench66_b$b.log | cut -c90-190)"
done
python - <<'PY'
import torch
print("device mem GB", torch.cuda.get_device_properties(0).total_memory / 2**30)
PY
