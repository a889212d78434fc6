#!/bin/bash
# Round 3, GPU pass 7: what limits the fused 1x1 GEMMs? Ablations of the quad-phase kernel and
# PMC passes (one counter group per run) on l3.0_down_dx for quad (mode 3) and conv1x1.hip (0);
# then the convergence comparison on a harder task (noise 4, 100 classes).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r03_07_*
timeout -k 10 300 python -u tools/diag/quad_ablate.py > $O/r03_07_ablate.jsonl 2> $O/r03_07_ablate.err || { tail -20 $O/r03_07_ablate.err; exit 1; }
cat $O/r03_07_ablate.jsonl
cd /tmp && export TMPDIR=/tmp
pmc() {  # tag mode counters...
  local tag=$1 m=$2; shift 2
  timeout -s KILL 90 rocprofv3 --output-format csv --pmc "$@" -d $O/r03_07_pmc${tag}_m$m -o run -- python3 $R/tools/diag/quad_ablate.py --only l3.0_down_dx --loop 5 --mode $m > $O/r03_07_pmc${tag}_m$m.log 2>&1
}
for m in 3 0; do
  pmc A $m SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU || { echo "pmcA m$m failed"; tail -5 $O/r03_07_pmcA_m$m.log; exit 1; }
  pmc B $m SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA || { echo "pmcB m$m failed"; tail -5 $O/r03_07_pmcB_m$m.log; exit 1; }
  pmc C $m TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr || { echo "pmcC m$m failed"; tail -5 $O/r03_07_pmcC_m$m.log; exit 1; }
done
cd $R
python tools/pmc_summary.py $O/r03_07_pmcA_m3 $O/r03_07_pmcB_m3 $O/r03_07_pmcC_m3 > $O/r03_07_pmc_quad.md 2>&1; head -30 $O/r03_07_pmc_quad.md
python tools/pmc_summary.py $O/r03_07_pmcA_m0 $O/r03_07_pmcB_m0 $O/r03_07_pmcC_m0 > $O/r03_07_pmc_old.md 2>&1; head -30 $O/r03_07_pmc_old.md
timeout -k 10 600 python -u bench/convergence.py --steps 100 --batch 128 --classes 100 --noise 4 --out $O/r03_07_conv > $O/r03_07_conv.log 2>&1 || { tail -30 $O/r03_07_conv.log; exit 1; }
tail -2 $O/r03_07_conv.log
