#!/bin/bash
# r06 pass 13: BN apply-pass grid cap A/B (CML_BN_GRID_CAP 2048 = grid-stride, 0 = one pass) on
# the headline step, alternating; BN tests with the one-pass grid.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_13; mkdir -p $O
cd $R
CML_BN_GRID_CAP=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_bn_gpu.py tests/test_kernels_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for cap in 2048 0 2048 0 16384; do
  CML_BN_GRID_CAP=$cap timeout -k 10 500 python -u bench.py --steps 10 --warmup 5 --no-baseline --b256-batch 0 --virtual-workers 0 > $O/b_$cap.json 2> $O/b_$cap.err || { tail -20 $O/b_$cap.err; exit 1; }
  python3 -c "
import json
r=json.loads([l for l in open('$O/b_$cap.json') if l.startswith('{')][0])
print('cap $cap', r['value'], r['ms_per_step'])"
done
for cap in 2048 0; do
  CML_AGG_GRID_CAP=$cap timeout -k 10 300 python -u bench/agg_kernels.py > $O/agg_$cap.jsonl 2> $O/agg_$cap.err || { tail -20 $O/agg_$cap.err; exit 1; }
  echo "agg cap $cap"; cut -c1-260 $O/agg_$cap.jsonl | head -4
done
for v in def zero def zero; do
  if [ $v = zero ]; then export CML_AGG_GRID_CAP=0 CML_GOSSIP_GRID_CAP=0 CML_STREAM_GRID_CAP=0; else unset CML_AGG_GRID_CAP CML_GOSSIP_GRID_CAP CML_STREAM_GRID_CAP; fi
  timeout -k 10 600 python -u bench/configs.py --config llama_gossip --loopback --steps 4 --warmup 2 --no-baseline --json-out $O/llama_$v.jsonl > $O/llama_$v.log 2>&1 || { tail -30 $O/llama_$v.log; exit 1; }
  python3 -c "import json; r=json.loads(open('$O/llama_$v.jsonl').readline()); print('llama $v', r['ms_per_step'])"
done
