#!/bin/bash
# r06 pass 26: the full GPU test suite after the stem / downsample / flash-width changes (as the driver runs it) + smoke().
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_26; mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -4 $O/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
