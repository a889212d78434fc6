#!/bin/bash
# Round 4, GPU pass 31: HBM bytes per step of the final round-4 code (rocprofv3 --pmc FETCH_SIZE /
# WRITE_SIZE, one counter per run, batch 2048): per class and per kernel group.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04_31}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --output-format csv --pmc $c -d $O/pmc_$c -o run -- python3 $R/bench.py --steps 3 --warmup 2 --no-baseline --b256-batch 0 --virtual-workers 0 --profile-marker > $O/pmc_$c.log 2>&1 || { tail -20 $O/pmc_$c.log; exit 1; }
  find $O/pmc_$c -type f ! -name 'run_counter_collection.csv' -delete
done
python3 $R/tools/pmc_step_bytes.py --steps 3 $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE > $O/step_bytes_b2048.md
python3 $R/tools/pmc_step_bytes.py --steps 3 --per-kernel 40 $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE > $O/step_bytes_per_kernel.md
cat $O/step_bytes_b2048.md
rm -rf $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE
