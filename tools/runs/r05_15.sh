#!/bin/bash
# r05 pass 15: stride-2 3x3 weight gradient on the wgrad DMA kernel: tests, per-shape bench,
# step A/B (own vs MIOpen stride-2 wgrad).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_15; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wgrad3x3s2_gpu.py tests/test_wgrad1x1_gpu.py > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -2 $O/test.log
timeout -k 10 300 python -u bench/wgrad_lib.py 2048 > $O/wgrad_lib.jsonl 2> $O/wgrad_lib.err || { tail -20 $O/wgrad_lib.err; exit 1; }
cat $O/wgrad_lib.jsonl
for rep in 1 2; do
for s2 in 0 1; do
CML_WGRAD3X3_S2=$s2 timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-baseline --b256-batch 0 --virtual-workers 0 > $O/bench_${s2}_${rep}.log 2>&1 || { tail -20 $O/bench_${s2}_${rep}.log; exit 1; }
echo "s2=$s2 rep=$rep $(grep '^{' $O/bench_${s2}_${rep}.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done
done
