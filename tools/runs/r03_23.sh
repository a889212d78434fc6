#!/bin/bash
# Round 3, GPU pass 23: tests that switch fusions through PerfPolicy scopes (they set module flags
# that no longer existed since the PerfPolicy refactor), then the full GPU suite, smoke, default bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r03_23_*
timeout -k 10 600 python -u -m pytest -q --timeout 180 --timeout-method thread -p no:cacheprovider tests/test_bn_gpu.py tests/test_stem_gpu.py tests/test_wgrad1x1_gpu.py tests/test_conv1x1_bn_gpu.py tests/test_transformer_ops_gpu.py > $O/r03_23_switch_tests.txt 2>&1; rc=$?
tail -15 $O/r03_23_switch_tests.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > $O/r03_23_gputests.txt 2>&1 || { tail -40 $O/r03_23_gputests.txt; exit 1; }
tail -3 $O/r03_23_gputests.txt
