#!/bin/bash
# r05 pass 36: conv_mm's sub-128-tile GEMMs (batch-256 layer 4) on gemm128.hip: tests, b256 step A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_36; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_mm_gpu.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
run() {   # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --batch 256 --steps 60 --warmup 10 --no-baseline --b256-batch 0 --virtual-workers 0 > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  echo "$tag $(grep '^{' $O/$tag.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
}
for rep in 1 2; do
run g128_$rep CML_OWN_GEMM128=1
run blas_$rep CML_OWN_GEMM128=0
done
