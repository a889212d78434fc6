#!/bin/bash
# r06 pass 23: stem_wgrad_pc_kernel with unconditional (clamped) producer prefetch and grouped
# input-tile loads: stem tests, ablations (1 no staging compute, 2 no products, 4 no restage),
# pc vs alternating microbench, ResNet A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_23; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_stem_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for a in 0 1 2 4 3; do
  CML_STEM_PC_ABL=$a timeout -k 10 200 python -u bench/stem_bwd.py --batch 2560 > $O/abl_$a.txt 2>&1 || { tail -20 $O/abl_$a.txt; exit 1; }
  echo "abl $a $(tail -1 $O/abl_$a.txt | cut -c1-100)"
done
for c in 1 0 1 0; do
  CML_STEM_PC=$c timeout -k 10 200 python -u bench/stem_bwd.py --batch 2560 > $O/stem_$c.txt 2>&1 || { tail -20 $O/stem_$c.txt; exit 1; }
  echo "pc $c $(tail -1 $O/stem_$c.txt)"
done
for c in 1 0 1 0; do
  CML_STEM_PC=$c timeout -k 10 500 python -u bench.py --steps 10 --warmup 5 --no-baseline --b256-batch 0 --virtual-workers 0 > $O/b_$c.json 2> $O/b_$c.err || { tail -20 $O/b_$c.err; exit 1; }
  python3 -c "
import json
r=json.loads([l for l in open('$O/b_$c.json') if l.startswith('{')][0])
print('resnet pc $c', r['value'], r['ms_per_step'])"
done
