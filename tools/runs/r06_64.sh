#!/bin/bash
# r06 pass 64: layer-1.0 conv1 data gradient (+ the downsample's dX) on the fused 1x1 kernel
# (conv1x1_link, no mask) instead of hipBLASLt: tests, A/B at batch 2560, library-kernel check.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_64; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  tests/test_fin_affine_gpu.py tests/test_stem_gpu.py tests/test_bwd_fusion_gpu.py tests/test_conv1x1g_gpu.py \
  tests/test_convergence_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  for f in 1 0; do
    CML_LINK_DGRAD_PLAIN=$f timeout -k 10 300 python3 bench.py --steps 20 --warmup 4 --no-baseline --b256-batch 0 \
      --virtual-workers 0 > $O/ab_${f}_$i.log 2>&1 || { tail -20 $O/ab_${f}_$i.log; exit 1; }
    echo "plain=$f run $i: $(grep '^{' $O/ab_${f}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
