#!/bin/bash
# GPU pass 16: transformer-op tests, BERT / Llama configs, steady-state profiles of both.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_transformer_ops_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_tops16.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_tops16.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench/configs.py --config bert_geomed --virtual-workers 8 --batch 32 --steps 10 --warmup 3 --json-out gpurun_out/configs16.jsonl > gpurun_out/configs16_bert.log 2>&1; rc=$?
tail -1 gpurun_out/configs16_bert.log | cut -c1-500
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench/configs.py --config llama_gossip --steps 5 --warmup 2 --json-out gpurun_out/configs16.jsonl > gpurun_out/configs16_llama.log 2>&1; rc=$?
tail -1 gpurun_out/configs16_llama.log | cut -c1-500
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
prof() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t rocprofv3 --kernel-trace -d $R/gpurun_out/raw_$name -o run -- "$@" > $R/gpurun_out/$name.log 2>&1 || return $?
  local db; db=$(find $R/gpurun_out/raw_$name -name '*.db' -print -quit)
  python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps $STEPS --top 45 --out $R/gpurun_out/${name}_kernels.md
  rm -rf $R/gpurun_out/raw_$name
}
STEPS=4 prof prof16_bert 300 python3 $R/bench/configs.py --config bert_geomed --virtual-workers 8 --batch 32 --steps 4 --warmup 2 --profile-marker || exit $?
STEPS=3 prof prof16_llama 400 python3 $R/bench/configs.py --config llama_gossip --steps 3 --warmup 2 --profile-marker || exit $?
