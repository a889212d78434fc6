#!/bin/bash
# r06 pass 27: Llama-3-8B with the w13 forward on gemm.hip (own forward up to 128 M weight
# elements, K <= 8192) vs the previous 32 M limit; transformer tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_27; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_transformer_ops_gpu.py tests/test_direct_grads_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for m in 134217728 33554432 134217728 33554432; do
  rm -f $O/llama_$m.jsonl
  CML_NB_OWN_FWD_MAX=$m timeout -k 10 600 python -u bench/configs.py --config llama_gossip --loopback --steps 4 --warmup 2 --no-baseline --json-out $O/llama_$m.jsonl > $O/llama_$m.log 2>&1 || { tail -30 $O/llama_$m.log; exit 1; }
  python3 -c "import json; r=json.loads(open('$O/llama_$m.jsonl').readline()); print('llama fwdmax $m', r['ms_per_step'])"
done
