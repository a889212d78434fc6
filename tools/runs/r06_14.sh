#!/bin/bash
# r06 pass 14: nontemporal loads in the BN passes (CML_BN_NT) A/B on the headline step; BN tests
# with NT on; the agg / gossip one-pass grids now default.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_14; mkdir -p $O
cd $R
CML_BN_NT=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_bn_gpu.py tests/test_kernels_gpu.py tests/test_agg_multi_gpu.py tests/test_gossip_graphs.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for nt in 0 1 0 1; do
  CML_BN_NT=$nt timeout -k 10 500 python -u bench.py --steps 10 --warmup 5 --no-baseline --b256-batch 0 --virtual-workers 0 > $O/b_$nt.json 2> $O/b_$nt.err || { tail -20 $O/b_$nt.err; exit 1; }
  python3 -c "
import json
r=json.loads([l for l in open('$O/b_$nt.json') if l.startswith('{')][0])
print('nt $nt', r['value'], r['ms_per_step'])"
done
