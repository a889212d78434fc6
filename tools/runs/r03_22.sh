#!/bin/bash
# Round 3, GPU pass 22: fresh-box confirmation of the round-3 code: the full GPU test suite,
# smoke(), the default bench line (as the driver runs it), BERT-base geomed 8 x 32 and Llama-3-8B
# gossip configs, aggregation kernel bandwidths.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r03_22_*
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > $O/r03_22_gputests.txt 2>&1 || { tail -40 $O/r03_22_gputests.txt; exit 1; }
tail -3 $O/r03_22_gputests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r03_22_smoke.txt 2>&1 || { tail -20 $O/r03_22_smoke.txt; exit 1; }
tail -1 $O/r03_22_smoke.txt
timeout -k 10 600 python -u bench.py > $O/r03_22_bench.log 2>&1 || { tail -30 $O/r03_22_bench.log; exit 1; }
grep '"metric"' $O/r03_22_bench.log > $O/r03_22_bench.json; cut -c1-600 $O/r03_22_bench.json
timeout -k 10 300 python -u bench/configs.py --config bert_geomed --virtual-workers 8 --batch 32 --steps 10 --warmup 3 --json-out $O/r03_22_bert.json > $O/r03_22_bert.log 2>&1 || { tail -20 $O/r03_22_bert.log; exit 1; }
cut -c1-400 $O/r03_22_bert.json
timeout -k 10 600 python -u bench/configs.py --config llama_gossip --steps 5 --warmup 2 --json-out $O/r03_22_llama.json > $O/r03_22_llama.log 2>&1 || { tail -20 $O/r03_22_llama.log; exit 1; }
cut -c1-400 $O/r03_22_llama.json
timeout -k 10 300 python -u bench/agg_kernels.py --json-out $O/r03_22_agg.jsonl > $O/r03_22_agg.log 2>&1 || { tail -20 $O/r03_22_agg.log; exit 1; }
cut -c1-300 $O/r03_22_agg.jsonl
