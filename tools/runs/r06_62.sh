#!/bin/bash
# r06 pass 62: cached 1x1 transposes only on the own-GEMM data-gradient path: ResNet tests + bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_62; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  tests/test_bwd_fusion_gpu.py tests/test_fin_affine_gpu.py tests/test_stem_gpu.py tests/test_side_wgrad_gpu.py \
  tests/test_conv_mm_gpu.py tests/test_convergence_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 4 --no-baseline --b256-batch 0 --virtual-workers 0 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])'
