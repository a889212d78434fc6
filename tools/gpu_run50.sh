#!/bin/bash
# GPU pass 50: full GPU test suite + smoke() after the stem kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest50.log 2>&1; rc=$?
tail -5 gpurun_out/pytest50.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke50.log 2>&1; rc=$?
tail -3 gpurun_out/smoke50.log
exit $rc
