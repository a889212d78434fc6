#!/bin/bash
# r05 pass 2: GPU tests touched by the engine / weights / gemm changes, then the headline bench
# (b256 early Grams) and the Llama-3-8B gossip config on the own flash attention.
set -o pipefail
mkdir -p gpurun_out/r05_02
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_weights_guard.py tests/test_gram_precision_gpu.py tests/test_engine_gpu.py \
  tests/test_loopback.py tests/test_transformer_ops_gpu.py tests/test_ffn_gpu.py \
  tests/test_gemm_gpu.py tests/test_kernels_gpu.py > gpurun_out/r05_02/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r05_02/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/r05_02/bench.json 2> gpurun_out/r05_02/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench/configs.py --config llama_gossip --steps 4 --warmup 2 --no-baseline \
  --json-out gpurun_out/r05_02/llama.jsonl > gpurun_out/r05_02/llama.out 2> gpurun_out/r05_02/llama.err
echo "llama rc=$?"
