#!/bin/bash
# GPU pass 62: own 1x1 weight gradient on all >=128-channel shapes vs the five core shapes vs off.
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in all core off all core off; do
  if [ $v = off ]; then export CML_WGRAD1X1=0; else export CML_WGRAD1X1=1 CML_WGRAD1X1_SET=$v; fi
  timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-baseline --json-out gpurun_out/bench62_$v.json > gpurun_out/bench62_$v.log 2>&1 || exit $?
  echo "$v $(tail -1 gpurun_out/bench62_$v.log | cut -c90-160)"
done
