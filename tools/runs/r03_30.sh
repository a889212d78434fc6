#!/bin/bash
# Round 3, GPU pass 30 (fresh container, HEAD re-validation): full GPU suite, stem gather-vs-two-pass-vs-fp64
# diagnosis, default bench line, step A/B (stem pool gather on / off), batch-256 kernel profile.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r03_30_*
timeout -k 10 900 python -u -m pytest tests -m gpu --deselect tests/test_convergence_gpu.py::test_fused_step_trains_like_library -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > $O/r03_30_gputests.txt 2>&1 || { tail -40 $O/r03_30_gputests.txt; exit 1; }
tail -2 $O/r03_30_gputests.txt
timeout -k 10 400 python -u tools/diag/stem_gather_diag.py > $O/r03_30_diag.jsonl 2>&1 || { tail -30 $O/r03_30_diag.jsonl; exit 1; }
grep '^{' $O/r03_30_diag.jsonl
timeout -k 10 600 python -u bench.py > $O/r03_30_bench.log 2>&1 || { tail -30 $O/r03_30_bench.log; exit 1; }
grep '"metric"' $O/r03_30_bench.log > $O/r03_30_bench.json; cut -c1-400 $O/r03_30_bench.json
for arm in default nogather; do
  case $arm in
    default) envs="";;
    nogather) envs="CML_STEM_POOL_GATHER=0";;
  esac
  env $envs timeout -k 10 300 python -u bench.py --steps 10 --warmup 4 --no-baseline --virtual-workers 0 --b256-batch 0 > $O/r03_30_bench_$arm.log 2>&1 || { tail -20 $O/r03_30_bench_$arm.log; exit 1; }
  echo "$arm $(grep -o '"ms_per_step": [0-9.]*' $O/r03_30_bench_$arm.log | head -1)" | tee -a $O/r03_30_ab.txt
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r03_30_prof256 -o run -- python3 $R/bench.py --batch 256 --steps 10 --warmup 4 --no-baseline --virtual-workers 0 --b256-batch 0 > $O/r03_30_prof256.log 2>&1 || { tail -20 $O/r03_30_prof256.log; exit 1; }
echo done
