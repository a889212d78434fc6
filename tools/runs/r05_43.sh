#!/bin/bash
# r05 pass 43 (repeat of 42, 3x3 only, 4 pairs): 3x3 weight gradients on a side stream (PerfPolicy.side_wgrad): bit-identity test,
# step A/B (CML_SIDE_WGRAD), kernel overlap visible in the busy fraction.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_43; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_side_wgrad_gpu.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
run() {   # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-baseline --b256-batch 0 --virtual-workers 0 > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  echo "$tag $(grep '^{' $O/$tag.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
}
for rep in 1 2 3 4; do
run side_$rep CML_SIDE_WGRAD=1
run base_$rep CML_SIDE_WGRAD=0
done
