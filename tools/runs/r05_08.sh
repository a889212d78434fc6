#!/bin/bash
# r05 pass 8: the full GPU test suite (as the driver runs it) + smoke().
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_08; mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1
rc=$?; tail -3 $O/gputests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/gputests.log | head -20; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
