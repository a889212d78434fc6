#!/bin/bash
# r06 pass 28: feature-selection GPU tests after the XGBoost-arithmetic split search (exact and
# histogram trees, the reference-parity GPU cases).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_28; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 600 --timeout-method thread tests/test_select_gpu.py tests/test_reference_rdata_parity.py tests/test_reference_parity.py tests/test_hist_trees.py > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
exit $rc
