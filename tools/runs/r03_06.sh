#!/bin/bash
# Round 3, GPU pass 6: small-launch attribution (batch 256 ResNet-50, BERT 8 x 32), aggregation
# kernel bandwidths with the centered Gram pass, the 2-rank gloo rehearsal of the N > 1 bench path
# (b256 block), rocprof kernel stats of the default bench step.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r03_06_*
timeout -k 10 300 python -u tools/small_kernels.py --batch 256 --top 60 > $O/r03_06_small_b256.txt 2>&1 || { tail -30 $O/r03_06_small_b256.txt; exit 1; }
head -40 $O/r03_06_small_b256.txt
timeout -k 10 300 python -u tools/small_kernels.py --model bert_base --batch 32 --virtual-workers 8 --rule geomed --top 60 > $O/r03_06_small_bert.txt 2>&1 || { tail -30 $O/r03_06_small_bert.txt; exit 1; }
head -40 $O/r03_06_small_bert.txt
timeout -k 10 300 python -u bench/agg_kernels.py --json-out $O/r03_06_agg.jsonl > $O/r03_06_agg.log 2>&1 || { tail -30 $O/r03_06_agg.log; exit 1; }
cut -c1-400 $O/r03_06_agg.jsonl
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --dist-backend gloo --batch 256 --steps 3 --warmup 1 --b256-batch 64 --b256-steps 3 --virtual-workers 0 > $O/r03_06_gloo2.log 2>&1 || { tail -30 $O/r03_06_gloo2.log; exit 1; }
grep '"metric"' $O/r03_06_gloo2.log > $O/r03_06_gloo2.json
cut -c1-3000 $O/r03_06_gloo2.json
