#!/bin/bash
# r06 pass 50: bn_stats_gram with 16 channels per workgroup (CML_GRAM_NC 16 vs 8): tests, per-shape timing, batch-256 A/B.
# launches, batch-256 A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_50; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  tests/test_bwd_fusion_gpu.py tests/test_fin_affine_gpu.py tests/test_convergence_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for f in 16 8; do
  CML_GRAM_NC=$f PYTHONPATH=$R timeout -k 10 120 python -u tools/diag/stats_gram_bench.py > $O/sg_$f.jsonl 2>&1 || { tail -5 $O/sg_$f.jsonl; exit 1; }
  echo "nc=$f: $(grep '^{' $O/sg_$f.jsonl | python3 -c 'import json,sys; print([json.loads(l)["us_per_call"] for l in sys.stdin])')"
done
for i in 1 2; do
  for f in 16 8; do
    CML_GRAM_NC=$f timeout -k 10 300 python3 bench.py --batch 256 --steps 40 --warmup 8 \
      --no-baseline --b256-batch 0 > $O/ab_${f}_$i.log 2>&1 || { tail -20 $O/ab_${f}_$i.log; exit 1; }
    echo "nc=$f run $i: $(grep '^{' $O/ab_${f}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
