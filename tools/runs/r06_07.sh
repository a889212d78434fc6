#!/bin/bash
# r06 pass 7: headline step at per-GPU batch 2048 / 3072 / 4096 (same box, headline block only)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_07; mkdir -p $O
cd $R
for b in 2048 2560 2048 2560; do
  timeout -k 10 500 python -u bench.py --batch $b --steps 10 --warmup 5 --no-baseline --b256-batch 0 --virtual-workers 0 > $O/b$b.json 2> $O/b$b.err || { tail -20 $O/b$b.err; exit 1; }
  python3 -c "
import json
r=json.loads([l for l in open('$O/b$b.json') if l.startswith('{')][0])
print($b, r['value'], r['ms_per_step'], r.get('peak_mem_gib'))"
done
