set -o pipefail
O=gpurun_out/${OUT:-r04_05}; mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_ffn_gpu.py tests/test_batched_workers_gpu.py tests/test_transformer_ops_gpu.py > $O/pytest.log 2>&1 && \
timeout -k 10 300 python bench/gemm.py --json-out $O/gemm.jsonl > $O/gemm.log 2>&1 && \
timeout -k 10 300 python bench/configs.py --config bert_geomed --virtual-workers 8 --batch 32 --steps 10 --warmup 3 --json-out $O/bert_v8.jsonl > $O/bert.log 2>&1
