#!/bin/bash
# r06 pass 9: exhaustive MIOpen search of the convolutions MIOpen still runs at per-GPU batch 2560
# (seeded with the shipped db), then the headline step at 2560 on the new db vs the shipped one.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_09; mkdir -p $O
cd $R
timeout -k 10 900 python -u tools/miopen_tune.py --batch 2560 --mode search --budget 700 --db tuning/miopen --out $O/miopen --only 64x56x56x64x1x1x0 128x56x56x128x3x2x1 256x56x56x64x1x1x0 > $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
tail -5 $O/tune.log
for db in new shipped new; do
  if [ $db = new ]; then export MIOPEN_USER_DB_PATH=$O/miopen; else unset MIOPEN_USER_DB_PATH; fi
  timeout -k 10 500 python -u bench.py --batch 2560 --steps 10 --warmup 5 --no-baseline --b256-batch 0 --virtual-workers 0 > $O/b_$db.json 2> $O/b_$db.err || { tail -20 $O/b_$db.err; exit 1; }
  python3 -c "
import json
r=json.loads([l for l in open('$O/b_$db.json') if l.startswith('{')][0])
print('$db', r['value'], r['ms_per_step'])"
done
