set -o pipefail
O=gpurun_out/${OUT:-r04_03}; mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_gpu.py > $O/pytest_gemm.log 2>&1 && \
timeout -k 10 300 python bench/gemm.py --json-out $O/gemm.jsonl > $O/gemm.log 2>&1
