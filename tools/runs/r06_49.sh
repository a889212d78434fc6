#!/bin/bash
# r06 pass 49: bn_stats_gram in one launch (CML_STATS_GRAM_ONE): tests, per-shape timing one vs two
# launches, batch-256 A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_49; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  tests/test_bwd_fusion_gpu.py tests/test_fin_affine_gpu.py tests/test_convergence_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for f in 1 0; do
  CML_STATS_GRAM_ONE=$f PYTHONPATH=$R timeout -k 10 120 python -u tools/diag/stats_gram_bench.py > $O/sg_$f.jsonl 2>&1 || { tail -5 $O/sg_$f.jsonl; exit 1; }
  echo "one=$f: $(grep '^{' $O/sg_$f.jsonl | python3 -c 'import json,sys; print([json.loads(l)["us_per_call"] for l in sys.stdin])')"
done
for i in 1 2; do
  for f in 1 0; do
    CML_STATS_GRAM_ONE=$f timeout -k 10 300 python3 bench.py --batch 256 --steps 40 --warmup 8 \
      --no-baseline --b256-batch 0 > $O/ab_${f}_$i.log 2>&1 || { tail -20 $O/ab_${f}_$i.log; exit 1; }
    echo "one=$f run $i: $(grep '^{' $O/ab_${f}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
