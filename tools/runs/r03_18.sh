#!/bin/bash
# Round 3, GPU pass 18: conv_gemm.hip 512 x 64 tiles of 128-pixel waves (narrow variant 4) for the
# 64-channel 3x3 convs: bit-identity / oracle tests, per-variant timing, step A/B (CML_CONV_GEMM_NARROW).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r03_18_*
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gemm_narrow_gpu.py tests/test_bwd_fusion_gpu.py -k "narrow or conv_gemm or cat or tail" > $O/r03_18_tests.txt 2>&1 || { tail -40 $O/r03_18_tests.txt; exit 1; }
tail -2 $O/r03_18_tests.txt
timeout -k 10 300 python -u bench/conv3x3_narrow.py > $O/r03_18_narrow.jsonl 2> $O/r03_18_narrow.err || { tail -20 $O/r03_18_narrow.err; exit 1; }
cat $O/r03_18_narrow.jsonl
for t in v0 v4 v0b v4b; do
  v=${t:1:1}
  CML_CONV_GEMM_NARROW=$v timeout -k 10 300 python -u bench.py --steps 12 --warmup 4 --b256-batch 0 --no-baseline --virtual-workers 0 > $O/r03_18_$t.log 2>&1 || { tail -20 $O/r03_18_$t.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('$O/r03_18_$t.log') if l.startswith('{\"metric')][0]); print('$t', d['ms_per_step'], d['value'])" | tee -a $O/r03_18_ab.txt
done
