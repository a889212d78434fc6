#!/bin/bash
# Round 3, GPU pass 25 (convergence test against a perturbed-library noise floor first): the full GPU test suite,
# smoke(), the default bench line (as the driver runs it), BERT-base geomed 8 x 32 and Llama-3-8B
# gossip configs, aggregation kernel bandwidths.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r03_25_*
timeout -k 10 300 python -u -m pytest -s -q --timeout 280 --timeout-method thread -p no:cacheprovider tests/test_convergence_gpu.py > $O/r03_25_conv.txt 2>&1 || { tail -30 $O/r03_25_conv.txt; exit 1; }
grep -A1 "fused vs library" $O/r03_25_conv.txt | cut -c1-1500
timeout -k 10 1000 python -u -m pytest tests -m gpu --deselect tests/test_convergence_gpu.py::test_fused_step_trains_like_library -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > $O/r03_25_gputests.txt 2>&1 || { tail -40 $O/r03_25_gputests.txt; exit 1; }
tail -3 $O/r03_25_gputests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r03_25_smoke.txt 2>&1 || { tail -20 $O/r03_25_smoke.txt; exit 1; }
tail -1 $O/r03_25_smoke.txt
timeout -k 10 600 python -u bench.py > $O/r03_25_bench.log 2>&1 || { tail -30 $O/r03_25_bench.log; exit 1; }
grep '"metric"' $O/r03_25_bench.log > $O/r03_25_bench.json; cut -c1-600 $O/r03_25_bench.json
timeout -k 10 300 python -u bench/configs.py --config bert_geomed --virtual-workers 8 --batch 32 --steps 10 --warmup 3 --json-out $O/r03_25_bert.json > $O/r03_25_bert.log 2>&1 || { tail -20 $O/r03_25_bert.log; exit 1; }
cut -c1-400 $O/r03_25_bert.json
timeout -k 10 600 python -u bench/configs.py --config llama_gossip --steps 5 --warmup 2 --json-out $O/r03_25_llama.json > $O/r03_25_llama.log 2>&1 || { tail -20 $O/r03_25_llama.log; exit 1; }
cut -c1-400 $O/r03_25_llama.json
timeout -k 10 300 python -u bench/agg_kernels.py --json-out $O/r03_25_agg.jsonl > $O/r03_25_agg.log 2>&1 || { tail -20 $O/r03_25_agg.log; exit 1; }
cut -c1-300 $O/r03_25_agg.jsonl
