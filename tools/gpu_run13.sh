#!/bin/bash
# GPU pass 13: steady-state kernel profiles of the transformer configs (BERT-base geomed with 8
# virtual workers, Llama-3-8B gossip), summarised on the box (raw rocpd output is deleted).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
prof() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t rocprofv3 --kernel-trace -d $R/gpurun_out/raw_$name -o run -- "$@" > $R/gpurun_out/$name.log 2>&1 || return $?
  tail -1 $R/gpurun_out/$name.log | cut -c1-400
  local db; db=$(find $R/gpurun_out/raw_$name -name '*.db' -print -quit)
  python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps $STEPS --top 45 --out $R/gpurun_out/${name}_kernels.md
  rm -rf $R/gpurun_out/raw_$name
}
STEPS=4 prof prof13_bert 300 python3 $R/bench/configs.py --config bert_geomed --virtual-workers 8 --batch 32 --steps 4 --warmup 2 --profile-marker || exit $?
STEPS=3 prof prof13_llama 400 python3 $R/bench/configs.py --config llama_gossip --steps 3 --warmup 2 --profile-marker || exit $?
