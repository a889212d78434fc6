#!/bin/bash
# Round 2, GPU pass 52: wide split-K fold (per-shape A/B) and bn2's backward sums from the dy2 GEMM
# epilogue (conv1x1_cat_bnsums + bn_bwd_apply), bn1's from the 3x3 data gradient's epilogue
# (conv_gemm_bnsums): numerics, step A/B of the three toggles.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r02_52_*
timeout -k 10 400 python -u -m pytest tests/test_bwd_fusion_gpu.py tests/test_wgrad1x1_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/r02_52_pytest.log 2>&1 || { tail -40 $O/r02_52_pytest.log; exit 1; }
tail -1 $O/r02_52_pytest.log
CML_FOLD_WIDE_MIN=0 timeout -k 10 120 python -u bench/fold.py --json-out $O/r02_52_fold.jsonl > $O/r02_52_fold0.log 2>&1 || { tail -20 $O/r02_52_fold0.log; exit 1; }
timeout -k 10 120 python -u bench/fold.py --json-out $O/r02_52_fold.jsonl > $O/r02_52_fold1.log 2>&1 || { tail -20 $O/r02_52_fold1.log; exit 1; }
cat $O/r02_52_fold.jsonl
for cfg in "0 0 0" "32 0 0" "32 1 0" "32 1 1" "0 0 0" "32 0 0" "32 1 0" "32 1 1"; do
set -- $cfg
CML_FOLD_WIDE_MIN=$1 CML_CAT_BNSUMS=$2 CML_BN1_DGRAD_SUMS=$3 timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-baseline --virtual-workers 0 > $O/r02_52_bench_$1_$2_$3.log 2>&1 || { tail -20 $O/r02_52_bench_$1_$2_$3.log; exit 1; }
echo "fold_wide_min=$1 cat_bnsums=$2 bn1_dgrad_sums=$3 $(grep -o '"ms_per_step": [0-9.]*' $O/r02_52_bench_$1_$2_$3.log)"
done
