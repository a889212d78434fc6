#!/bin/bash
# Round 2, GPU pass 51: wide split-K fold (16 split lanes per 64 outputs) for slabs with >= 32
# splits: numerics, per-shape A/B against the narrow fold, step A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r02_51_*
timeout -k 10 300 python -u -m pytest tests/test_wgrad1x1_gpu.py tests/test_bwd_fusion_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/r02_51_pytest.log 2>&1 || { tail -40 $O/r02_51_pytest.log; exit 1; }
tail -1 $O/r02_51_pytest.log
CML_FOLD_WIDE_MIN=0 timeout -k 10 120 python -u bench/fold.py --json-out $O/r02_51_fold.jsonl > $O/r02_51_fold0.log 2>&1 || { tail -20 $O/r02_51_fold0.log; exit 1; }
timeout -k 10 120 python -u bench/fold.py --json-out $O/r02_51_fold.jsonl > $O/r02_51_fold1.log 2>&1 || { tail -20 $O/r02_51_fold1.log; exit 1; }
cat $O/r02_51_fold.jsonl
for f in 0 32 0 32; do
CML_FOLD_WIDE_MIN=$f timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-baseline --virtual-workers 0 > $O/r02_51_bench$f.log 2>&1 || { tail -20 $O/r02_51_bench$f.log; exit 1; }
echo "fold_wide_min=$f $(grep -o '"ms_per_step": [0-9.]*' $O/r02_51_bench$f.log)"
done
