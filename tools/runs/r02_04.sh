#!/bin/bash
# Round 2, GPU pass 4: fused conv+BN integrated into ResNet-50: numerics (kernel + whole model),
# full GPU suite, per-shape timing with the 128x128 fallback tile, default bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv1x1_bn_gpu.py -x -q --timeout 120 --timeout-method thread > $O/r02_04_pytest_conv.log 2>&1 || { tail -40 $O/r02_04_pytest_conv.log; exit 1; }
tail -2 $O/r02_04_pytest_conv.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/r02_04_pytest.log 2>&1 || { tail -40 $O/r02_04_pytest.log; exit 1; }
tail -2 $O/r02_04_pytest.log
timeout -k 10 300 python -u bench/conv1x1_fused.py --batch 2048 --json-out $O/r02_04_conv1x1.jsonl > $O/r02_04_convbench.log 2>&1 || { tail -20 $O/r02_04_convbench.log; exit 1; }
cut -c1-60,200-330 $O/r02_04_convbench.log
timeout -k 10 400 python -u bench.py > $O/r02_04_bench.log 2>&1 || { tail -20 $O/r02_04_bench.log; exit 1; }
tail -1 $O/r02_04_bench.log | cut -c1-900
