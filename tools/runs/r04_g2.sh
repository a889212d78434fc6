set -o pipefail
O=gpurun_out/r04_02; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gram_precision_gpu.py tests/test_engine_gpu.py > $O/pytest.log 2>&1 && \
timeout -k 10 300 python bench.py --loopback off --json-out $O/bench_n1_noloop.json > $O/bench_noloop.log 2>&1 && \
timeout -k 10 300 python bench.py --loopback on --json-out $O/bench_n1_loop.json > $O/bench_loop.log 2>&1 && \
timeout -k 10 300 python bench/gossip_mix.py --json-out $O/gossip_mix.jsonl > $O/gossip_mix.log 2>&1 && \
timeout -k 10 600 python bench/configs.py --config llama_gossip --loopback --steps 5 --warmup 2 --json-out $O/llama_gossip_loop.jsonl > $O/llama.log 2>&1
