#!/bin/bash
# Round 3, GPU pass 35 (final code of the round): convergence test, the full GPU suite, smoke(), the
# default bench line (as the driver runs it), a 2-rank gloo rehearsal of the N > 1 bench path,
# BERT-base geomed 8 x 32 and Llama-3-8B gossip configs.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r03_35_*
timeout -k 10 300 python -u -m pytest -s -q --timeout 280 --timeout-method thread -p no:cacheprovider tests/test_convergence_gpu.py > $O/r03_35_conv.txt 2>&1 || { tail -30 $O/r03_35_conv.txt; exit 1; }
grep -A1 "fused vs library" $O/r03_35_conv.txt | cut -c1-1500
timeout -k 10 900 python -u -m pytest tests -m gpu --deselect tests/test_convergence_gpu.py::test_fused_step_trains_like_library -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > $O/r03_35_gputests.txt 2>&1 || { tail -40 $O/r03_35_gputests.txt; exit 1; }
tail -2 $O/r03_35_gputests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r03_35_smoke.txt 2>&1 || { tail -20 $O/r03_35_smoke.txt; exit 1; }
tail -1 $O/r03_35_smoke.txt
timeout -k 10 600 python -u bench.py > $O/r03_35_bench.log 2>&1 || { tail -30 $O/r03_35_bench.log; exit 1; }
grep '"metric"' $O/r03_35_bench.log > $O/r03_35_bench.json; cut -c1-600 $O/r03_35_bench.json
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29635 bench.py --gpus 2 --dist-backend gloo --batch 256 --steps 3 --warmup 1 --b256-batch 64 --b256-steps 3 --virtual-workers 0 > $O/r03_35_gloo2.log 2>&1 || { tail -30 $O/r03_35_gloo2.log; exit 1; }
grep '"metric"' $O/r03_35_gloo2.log > $O/r03_35_gloo2.json; cut -c1-600 $O/r03_35_gloo2.json
timeout -k 10 300 python -u bench/configs.py --config bert_geomed --virtual-workers 8 --batch 32 --steps 10 --warmup 3 --json-out $O/r03_35_bert.json > $O/r03_35_bert.log 2>&1 || { tail -20 $O/r03_35_bert.log; exit 1; }
cut -c1-400 $O/r03_35_bert.json
timeout -k 10 600 python -u bench/configs.py --config llama_gossip --steps 5 --warmup 2 --json-out $O/r03_35_llama.json > $O/r03_35_llama.log 2>&1 || { tail -20 $O/r03_35_llama.log; exit 1; }
cut -c1-400 $O/r03_35_llama.json
