#!/bin/bash
# r05 pass 14: A/B of the LDS-DMA wgrad1x1 in the step (interleaved), own-set shapes per kernel.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_14; mkdir -p $O
cd $R
timeout -k 10 300 python -u bench/wgrad_lib.py 2048 --core > $O/wgrad_dma.jsonl 2> $O/wgrad_lib.err || { tail -20 $O/wgrad_lib.err; exit 1; }
CML_WGRAD_DMA=0 timeout -k 10 300 python -u bench/wgrad_lib.py 2048 --core > $O/wgrad_nodma.jsonl 2>> $O/wgrad_lib.err || { tail -20 $O/wgrad_lib.err; exit 1; }
tail -6 $O/wgrad_dma.jsonl; tail -6 $O/wgrad_nodma.jsonl
for rep in 1 2; do
for cfg in "0 core" "1 core" "1 wide"; do
set -- $cfg
CML_WGRAD_DMA=$1 CML_WGRAD1X1_SET=$2 timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-baseline --b256-batch 0 --virtual-workers 0 > $O/bench_$1_$2_$rep.log 2>&1 || { tail -20 $O/bench_$1_$2_$rep.log; exit 1; }
echo "dma=$1 set=$2 rep=$rep $(grep '^{' $O/bench_$1_$2_$rep.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done
done
