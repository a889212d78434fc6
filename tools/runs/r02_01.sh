#!/bin/bash
# Round 2, GPU pass 1: GPU tests after the ADVICE fixes, MIOpen find-db for batch 256 (virtual
# workers of the bench), then the default bench with the new virtual-worker Krum block.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/r02_01_pytest.log 2>&1 || { tail -30 $O/r02_01_pytest.log; exit 1; }
tail -3 $O/r02_01_pytest.log
timeout -k 10 900 python -u tools/miopen_tune.py --mode find --batch 256 --db tuning/miopen --out $O/miopen_b256 --budget 800 > $O/r02_01_tune.log 2>&1 || { tail -20 $O/r02_01_tune.log; exit 1; }
tail -2 $O/r02_01_tune.log
export MIOPEN_USER_DB_PATH=$O/miopen_b256
timeout -k 10 400 python -u bench.py > $O/r02_01_bench.log 2>&1 || { tail -20 $O/r02_01_bench.log; exit 1; }
tail -1 $O/r02_01_bench.log
