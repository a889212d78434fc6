#!/bin/bash
# r06 pass 3: gemm_w4 after retiring the previous fragment reads at the step start (no lgkmcnt(0)
# (CML_W4_ABL: 1 no staging, 2 no fragment reads, 4 no barrier, 7 none of them) at 8192^3.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_03; mkdir -p $O
cd $R
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_w4_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for sch in 1 2; do
  CML_W4_SCHED=$sch timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_w4_gpu.py > $O/tests_s$sch.log 2>&1 || { tail -40 $O/tests_s$sch.log; exit 1; }
  tail -1 $O/tests_s$sch.log
done
for sch in 0 2; do
  CML_W4_SCHED=$sch timeout -k 10 200 python -u bench/gemm_w4.py --only sq8k wo --ops fwd dgrad wgrad > $O/sch$sch.jsonl 2>&1 || { tail -20 $O/sch$sch.jsonl; exit 1; }
  echo "sched $sch"; cut -c1-250 $O/sch$sch.jsonl
done
for abl in 7; do
  CML_W4_ABL=$abl timeout -k 10 200 python -u bench/gemm_w4.py --only sq8k > $O/abl$abl.jsonl 2>&1 || { tail -20 $O/abl$abl.jsonl; exit 1; }
  echo "abl $abl"; cut -c1-200 $O/abl$abl.jsonl | head -1
done
