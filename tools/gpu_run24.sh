#!/bin/bash
# GPU pass 24: refresh the shipped MIOpen find-db for the current conv set (stem with 4 input
# channels, MIOpen weight gradients of the GEMM-forward 1x1 convs): run the bench once with find
# mode on, then copy the user db back.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export MIOPEN_USER_DB_PATH=/tmp/cml_miopen_db_refresh
mkdir -p $MIOPEN_USER_DB_PATH && cp tuning/miopen/*.txt $MIOPEN_USER_DB_PATH/
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --json-out gpurun_out/bench24.json > gpurun_out/bench24.log 2>&1; rc=$?
grep warmup gpurun_out/bench24.log
tail -1 gpurun_out/bench24.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
mkdir -p gpurun_out/miopen_db && cp $MIOPEN_USER_DB_PATH/*.txt gpurun_out/miopen_db/ && wc -l gpurun_out/miopen_db/*
