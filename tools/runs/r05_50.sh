#!/bin/bash
# r05 pass 50: a weight gradient's dW and column-sum folds in one launch: tests, b256 / b2048 steps.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_50; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_wgrad1x1_gpu.py tests/test_bwd_fusion_gpu.py tests/test_wgrad3x3s2_gpu.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-baseline --virtual-workers 0 > $O/step.log 2>&1 || { tail -20 $O/step.log; exit 1; }
grep '^{' $O/step.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("b256_ms_per_step"))'
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw -o run -- python3 $R/bench.py --batch 256 --steps 10 --warmup 5 --no-baseline --b256-batch 0 --virtual-workers 0 --profile-marker > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
db=$(find $O/raw -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 10 --top 400 --out $O/kernels_b256.md > /dev/null
rm -rf $O/raw
head -2 $O/kernels_b256.md
grep -E "fold" $O/kernels_b256.md | cut -c1-160
