#!/bin/bash
# Round 3, GPU pass 9: packed-VALU prologues (bnrelu_pk / mask_pk), the cat GEMMs' BN-backward
# affine folded into w + an epilogue bias, identity second sources. Fused-kernel tests, per-shape
# kernel families, quad ablation, default bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r03_09_*
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bwd_fusion_gpu.py tests/test_conv1x1g_gpu.py tests/test_conv1x1_bn_gpu.py > $O/r03_09_tests.txt 2>&1 || { tail -40 $O/r03_09_tests.txt; exit 1; }
tail -3 $O/r03_09_tests.txt
timeout -k 10 300 python -u bench/conv1x1g.py --json-out $O/r03_09_families.jsonl > $O/r03_09_families.log 2>&1 || { tail -30 $O/r03_09_families.log; exit 1; }
cut -c1-300 $O/r03_09_families.jsonl
timeout -k 10 300 python -u tools/diag/quad_ablate.py > $O/r03_09_ablate.jsonl 2> $O/r03_09_ablate.err || { tail -20 $O/r03_09_ablate.err; exit 1; }
cat $O/r03_09_ablate.jsonl
timeout -k 10 300 python -u bench.py --steps 10 --warmup 4 > $O/r03_09_bench.log 2>&1 || { tail -30 $O/r03_09_bench.log; exit 1; }
grep '"metric"' $O/r03_09_bench.log | cut -c1-700
