#!/bin/bash
# Round 2, GPU pass 66: fresh-box confirmation of the committed state: smoke, full GPU suite,
# default bench (batch 2048 + the 8 x 256 virtual-worker Krum block), batch-256 bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r02_66_*
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r02_66_smoke.log 2>&1 || { tail -30 $O/r02_66_smoke.log; exit 1; }
tail -1 $O/r02_66_smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r02_66_pytest.log 2>&1 || { tail -40 $O/r02_66_pytest.log; exit 1; }
tail -1 $O/r02_66_pytest.log
timeout -k 10 600 python -u bench.py > $O/r02_66_bench.log 2>&1 || { tail -20 $O/r02_66_bench.log; exit 1; }
grep '^{' $O/r02_66_bench.log > $O/r02_66_bench.json
cut -c1-400 $O/r02_66_bench.json
timeout -k 10 600 python -u bench.py --batch 256 --steps 50 --warmup 10 > $O/r02_66_bench256.log 2>&1 || { tail -20 $O/r02_66_bench256.log; exit 1; }
grep '^{' $O/r02_66_bench256.log > $O/r02_66_bench256.json
cut -c1-400 $O/r02_66_bench256.json
