#!/bin/bash
# GPU pass 64: full GPU suite + smoke + default bench (round-end rehearsal).
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest64.log 2>&1; rc=$?
tail -3 gpurun_out/pytest64.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke64.log 2>&1 || exit $?
tail -1 gpurun_out/smoke64.log
timeout -k 10 500 python bench.py > gpurun_out/bench64_default.log 2>&1 || exit $?
tail -1 gpurun_out/bench64_default.log | cut -c1-400
