#!/bin/bash
# r05 pass 16: the 128 x 128 stride-2 tile with 4 / 8 stages.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_16; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wgrad3x3s2_gpu.py > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -2 $O/test.log
for ns in 4 8; do
CML_WGRAD_DMA_NS128=$ns timeout -k 10 300 python -u bench/wgrad_lib.py 2048 > $O/wgrad_lib_ns$ns.jsonl 2> $O/wgrad_lib.err || { tail -20 $O/wgrad_lib.err; exit 1; }
grep '"k": 3' $O/wgrad_lib_ns$ns.jsonl
done
