#!/bin/bash
# Round 2, GPU pass 50: fresh-box confirmation after container re-creation: smoke, full GPU suite, default bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r02_50_*
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r02_50_smoke.log 2>&1 || { tail -30 $O/r02_50_smoke.log; exit 1; }
tail -1 $O/r02_50_smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r02_50_pytest.log 2>&1 || { tail -40 $O/r02_50_pytest.log; exit 1; }
tail -1 $O/r02_50_pytest.log
timeout -k 10 600 python -u bench.py > $O/r02_50_bench.log 2>&1 || { tail -20 $O/r02_50_bench.log; exit 1; }
grep '^{' $O/r02_50_bench.log > $O/r02_50_bench.json
cut -c1-600 $O/r02_50_bench.json
