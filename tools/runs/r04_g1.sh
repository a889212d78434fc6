set -o pipefail
mkdir -p gpurun_out/r04_01
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_loopback.py -m gpu > gpurun_out/r04_01/loopback.log 2>&1 && \
timeout -k 10 400 python bench.py --json-out gpurun_out/r04_01/bench_n1.json > gpurun_out/r04_01/bench_n1.log 2>&1 && \
timeout -k 10 400 python bench.py --gpus 8 --dist-backend gloo --batch 16 --image-size 64 --steps 3 --warmup 1 --no-miopen-find --b256-batch 0 --no-baseline --timeout 300 --json-out gpurun_out/r04_01/gloo8.json > gpurun_out/r04_01/gloo8.log 2>&1
