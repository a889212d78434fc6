#!/bin/bash
# GPU pass 25: PMC counters (FETCH_SIZE | WRITE_SIZE, one group per run, --kernel-trace --stats
# only) over the ResNet-50 bench step and the BERT config: HBM bytes per kernel for the fused BN,
# pooling, transformer and aggregation kernels. Raw output is summarised on the box and deleted.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
run_pmc() {  # tag, group, command...
  local tag=$1 grp=$2; shift 2
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --stats --output-format csv -d $R/gpurun_out/pmc25_$tag -o run -- "$@" > $R/gpurun_out/pmc25_$tag.log 2>&1 || return $?
  tail -1 $R/gpurun_out/pmc25_$tag.log | cut -c1-200
}
run_pmc resnet_fetch FETCH_SIZE python3 $R/bench.py --steps 2 --warmup 1 --no-baseline || exit $?
run_pmc resnet_write WRITE_SIZE python3 $R/bench.py --steps 2 --warmup 1 --no-baseline || exit $?
run_pmc bert_fetch FETCH_SIZE python3 $R/bench/configs.py --config bert_geomed --virtual-workers 8 --batch 32 --steps 1 --warmup 1 || exit $?
run_pmc bert_write WRITE_SIZE python3 $R/bench/configs.py --config bert_geomed --virtual-workers 8 --batch 32 --steps 1 --warmup 1 || exit $?
cd $R
python3 tools/pmc_summary.py gpurun_out/pmc25_resnet_fetch gpurun_out/pmc25_resnet_write > gpurun_out/pmc25_resnet.md || exit $?
python3 tools/pmc_summary.py gpurun_out/pmc25_bert_fetch gpurun_out/pmc25_bert_write > gpurun_out/pmc25_bert.md || exit $?
find gpurun_out/pmc25_* -maxdepth 0 -type d -exec rm -rf {} +
head -30 gpurun_out/pmc25_resnet.md | cut -c1-200
