#!/bin/bash
# r06 pass 55: 1x1 weight gradients on the side stream too (CML_SIDE_WGRAD_1X1): side-stream tests,
# batch-2560 A/B (1x1 + 3x3 on the side stream vs 3x3 only), alternating.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_55; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  tests/test_side_wgrad_gpu.py tests/test_fin_affine_gpu.py tests/test_convergence_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  for f in 1 0; do
    CML_SIDE_WGRAD_1X1=$f timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-baseline --b256-batch 0 \
      --virtual-workers 0 > $O/b2560_${f}_$i.log 2>&1 || { tail -20 $O/b2560_${f}_$i.log; exit 1; }
    echo "b2560 side1x1=$f run $i: $(grep '^{' $O/b2560_${f}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
