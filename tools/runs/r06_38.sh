#!/bin/bash
# r06 pass 38: flash forward / dQ with 8-wave workgroups by default: flash tests, the Llama step
# vs 4-wave (CML_FA_WAVES=4).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_38; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_flash_attn_gpu.py tests/test_transformer_ops_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for wv in 8 4 8 4; do
  rm -f $O/llama_$wv.jsonl
  CML_FA_WAVES=$wv timeout -k 10 600 python -u bench/configs.py --config llama_gossip --loopback --steps 4 --warmup 2 --no-baseline --json-out $O/llama_$wv.jsonl > $O/llama_$wv.log 2>&1 || { tail -30 $O/llama_$wv.log; exit 1; }
  python3 -c "import json; r=json.loads(open('$O/llama_$wv.jsonl').readline()); print('llama waves $wv', r['ms_per_step'])"
done
