#!/bin/bash
# r05 pass 35: HBM rates; conv_mm GEMMs on the 256 vs 128 tile vs hipBLASLt (batch 2048 / 256).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_35; mkdir -p $O
cd $R
timeout -k 10 300 python -u bench/hbm_rates.py > $O/hbm.jsonl 2> $O/hbm.err || { tail -20 $O/hbm.err; exit 1; }
cat $O/hbm.jsonl
for b in 2048 256; do
timeout -k 10 300 python -u bench/conv_mm_tiles.py --batch $b > $O/conv_mm_b$b.jsonl 2> $O/conv_mm_b$b.err || { tail -20 $O/conv_mm_b$b.err; exit 1; }
cat $O/conv_mm_b$b.jsonl
done
