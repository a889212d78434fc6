#!/bin/bash
# GPU pass 72: full GPU suite + smoke + default bench (final round-end rehearsal).
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest72.log 2>&1; rc=$?
tail -3 gpurun_out/pytest72.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke72.log 2>&1 || exit $?
tail -1 gpurun_out/smoke72.log
