#!/bin/bash
# r06 pass 29: BN apply-pass grid cap sweep on the ResNet step (CML_BN_GRID_CAP; 2048 default).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_29; mkdir -p $O
cd $R
for c in 2048 8192 4096 16384 2048 8192 4096 16384; do
  CML_BN_GRID_CAP=$c timeout -k 10 500 python -u bench.py --steps 10 --warmup 5 --no-baseline --b256-batch 0 --virtual-workers 0 > $O/b_$c.json 2> $O/b_$c.err || { tail -20 $O/b_$c.err; exit 1; }
  python3 -c "
import json
r=json.loads([l for l in open('$O/b_$c.json') if l.startswith('{')][0])
print('resnet bn cap $c', r['value'], r['ms_per_step'])"
done
