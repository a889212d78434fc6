#!/bin/bash
# GPU pass 6: tests (maxpool), counter list, MIOpen find-db capture (batch 512), agg kernel
# micro-bench + PMC counters.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/miopen_db gpurun_out/miopen_cache2
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1 || true
export MIOPEN_USER_DB_PATH=$GRAFT_REPO_ROOT/gpurun_out/miopen_db
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --batch 512 --no-baseline > gpurun_out/bench6_cold.log 2>&1; rc=$?
tail -2 gpurun_out/bench6_cold.log
[ $rc -eq 0 ] || exit $rc
MIOPEN_CUSTOM_CACHE_DIR=$GRAFT_REPO_ROOT/gpurun_out/miopen_cache2 timeout -k 10 400 python bench.py --steps 20 --warmup 3 --batch 512 --no-baseline > gpurun_out/bench6_warmdb.log 2>&1; rc=$?
tail -2 gpurun_out/bench6_warmdb.log
rm -rf gpurun_out/miopen_cache2
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench/agg_kernels.py --json-out gpurun_out/agg_kernels6.jsonl > gpurun_out/agg6.log 2>&1; rc=$?
tail -6 gpurun_out/agg6.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE GRBM_GUI_ACTIVE --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc6a -o run -- python3 $GRAFT_REPO_ROOT/bench/agg_kernels.py --n 8 --D 25557032 --reps 3 --no-torch > $GRAFT_REPO_ROOT/gpurun_out/pmc6a.log 2>&1; rc=$?
tail -3 $GRAFT_REPO_ROOT/gpurun_out/pmc6a.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc6b -o run -- python3 $GRAFT_REPO_ROOT/bench/agg_kernels.py --n 8 --D 25557032 --reps 3 --no-torch > $GRAFT_REPO_ROOT/gpurun_out/pmc6b.log 2>&1; rc=$?
tail -3 $GRAFT_REPO_ROOT/gpurun_out/pmc6b.log
exit 0
