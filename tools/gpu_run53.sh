#!/bin/bash
# GPU pass 53: bench A/B — shipped find-db vs the exhaustively searched one (tools/miopen_tune.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p /tmp/db_search && cp tuning/miopen_search/*.udb.txt tuning/miopen_search/*.ufdb.txt /tmp/db_search/
for v in old new old new; do
  if [ $v = new ]; then export MIOPEN_USER_DB_PATH=/tmp/db_search; else unset MIOPEN_USER_DB_PATH; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-baseline --json-out gpurun_out/bench53_$v.json > gpurun_out/bench53_$v.log 2>&1 || exit $?
  echo "$v $(tail -1 gpurun_out/bench53_$v.log | cut -c90-170)"
done
