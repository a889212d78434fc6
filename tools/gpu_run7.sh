#!/bin/bash
# GPU pass 7: tests (packed-key sort, packed Gram), agg kernel micro-bench, headline bench with the
# shipped MIOpen find-db, PMC counters in single-group passes, reference timings.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu7.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu7.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench/agg_kernels.py --n 1 2 4 8 16 32 --json-out gpurun_out/agg_kernels7.jsonl > gpurun_out/agg7.log 2>&1; rc=$?
tail -8 gpurun_out/agg7.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python bench.py --steps 20 --warmup 3 --json-out gpurun_out/bench7.json > gpurun_out/bench7.log 2>&1; rc=$?
tail -2 gpurun_out/bench7.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof7 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof7.log 2>&1; rc=$?
tail -2 $GRAFT_REPO_ROOT/gpurun_out/prof7.log
[ $rc -eq 0 ] || exit $rc
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES"; do
  tag=$(echo $grp | cut -d' ' -f1 | tr 'A-Z' 'a-z')
  timeout -k 10 180 rocprofv3 --pmc $grp --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc7_$tag -o run -- python3 $GRAFT_REPO_ROOT/bench/agg_kernels.py --n 8 --D 25557032 --reps 3 --no-torch > $GRAFT_REPO_ROOT/gpurun_out/pmc7_$tag.log 2>&1; rc=$?
  tail -2 $GRAFT_REPO_ROOT/gpurun_out/pmc7_$tag.log
  [ $rc -eq 0 ] || exit $rc
done
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python bench/reference_timings.py > gpurun_out/reftime7.log 2>&1; rc=$?
tail -5 gpurun_out/reftime7.log
exit $rc
