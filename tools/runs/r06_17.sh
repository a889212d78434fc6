#!/bin/bash
# r06 pass 17: Llama step with own wqkv / wo forwards and own w2 data gradients (gemm.hip grouped
# order), alternating with the gemm.hip round-5 order (CML_GEMM_GM=0); ResNet headline A/B of the
# grouped order (its 1x1 GEMMs); the transformer GPU tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_17; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_transformer_ops_gpu.py tests/test_direct_grads_gpu.py tests/test_gemm_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for gm in 8 0 8 0; do
  CML_GEMM_GM=$gm timeout -k 10 500 python -u bench.py --steps 10 --warmup 5 --no-baseline --b256-batch 0 --virtual-workers 0 > $O/b_$gm.json 2> $O/b_$gm.err || { tail -20 $O/b_$gm.err; exit 1; }
  python3 -c "
import json
r=json.loads([l for l in open('$O/b_$gm.json') if l.startswith('{')][0])
print('resnet gm $gm', r['value'], r['ms_per_step'])"
done
for gm in 8 0 8; do
  rm -f $O/llama_$gm.jsonl
  CML_GEMM_GM=$gm timeout -k 10 600 python -u bench/configs.py --config llama_gossip --loopback --steps 4 --warmup 2 --no-baseline --json-out $O/llama_$gm.jsonl > $O/llama_$gm.log 2>&1 || { tail -30 $O/llama_$gm.log; exit 1; }
  python3 -c "import json; r=json.loads(open('$O/llama_$gm.jsonl').readline()); print('llama gm $gm', r['ms_per_step'], r.get('phase_ms_per_step'))"
done
