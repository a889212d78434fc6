#!/bin/bash
# GPU pass 15: BERT-base steady-state kernel profile with the fused transformer kernels.
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
STEPS=4 prof prof15_bert 300 python3 $R/bench/configs.py --config bert_geomed --virtual-workers 8 --batch 32 --steps 4 --warmup 2 --profile-marker || exit $?
