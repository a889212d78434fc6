#!/bin/bash
# r06 pass 30: layer-1.0 conv1 (64 -> 64) data gradient as a GEMM absorbing the downsample's dX
# (CML_C1_DGRAD64=1) vs MIOpen + the stem pool backward's two-gradient sum; ResNet A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_30; mkdir -p $O
cd $R
for c in 1 0 1 0; do
  CML_C1_DGRAD64=$c timeout -k 10 500 python -u bench.py --steps 10 --warmup 5 --no-baseline --b256-batch 0 --virtual-workers 0 > $O/b_$c.json 2> $O/b_$c.err || { tail -20 $O/b_$c.err; exit 1; }
  python3 -c "
import json
r=json.loads([l for l in open('$O/b_$c.json') if l.startswith('{')][0])
print('resnet dgrad64 $c', r['value'], r['ms_per_step'])"
done
