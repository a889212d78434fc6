#!/bin/bash
# Round 3, GPU pass 8 (re-run of passes 6-7 whose outputs were lost with the container):
# small-launch attribution (batch 256 ResNet-50, BERT 8 x 32), the 2-rank gloo rehearsal of the
# N > 1 bench path (b256 block), quad-kernel ablations + PMC passes on l3.0_down_dx, default bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r03_08_*
timeout -k 10 300 python -u tools/small_kernels.py --batch 256 --top 60 > $O/r03_08_small_b256.txt 2>&1 || { tail -30 $O/r03_08_small_b256.txt; exit 1; }
head -30 $O/r03_08_small_b256.txt
timeout -k 10 300 python -u tools/small_kernels.py --model bert_base --batch 32 --virtual-workers 8 --rule geomed --top 60 > $O/r03_08_small_bert.txt 2>&1 || { tail -30 $O/r03_08_small_bert.txt; exit 1; }
head -30 $O/r03_08_small_bert.txt
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --dist-backend gloo --batch 256 --steps 3 --warmup 1 --b256-batch 64 --b256-steps 3 --virtual-workers 0 > $O/r03_08_gloo2.log 2>&1 || { tail -30 $O/r03_08_gloo2.log; exit 1; }
grep '"metric"' $O/r03_08_gloo2.log > $O/r03_08_gloo2.json
cut -c1-2000 $O/r03_08_gloo2.json
timeout -k 10 300 python -u tools/diag/quad_ablate.py > $O/r03_08_ablate.jsonl 2> $O/r03_08_ablate.err || { tail -20 $O/r03_08_ablate.err; exit 1; }
cat $O/r03_08_ablate.jsonl
cd /tmp && export TMPDIR=/tmp
pmc() {  # tag mode counters...
  local tag=$1 m=$2; shift 2
  timeout -s KILL 90 rocprofv3 --output-format csv --pmc "$@" -d $O/r03_08_pmc${tag}_m$m -o run -- python3 $R/tools/diag/quad_ablate.py --only l3.0_down_dx --loop 5 --mode $m > $O/r03_08_pmc${tag}_m$m.log 2>&1
}
for m in 3 0; do
  pmc A $m SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU || { echo "pmcA m$m failed"; tail -5 $O/r03_08_pmcA_m$m.log; exit 1; }
  pmc B $m SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA || { echo "pmcB m$m failed"; tail -5 $O/r03_08_pmcB_m$m.log; exit 1; }
  pmc C $m TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr || { echo "pmcC m$m failed"; tail -5 $O/r03_08_pmcC_m$m.log; exit 1; }
done
cd $R
python tools/pmc_summary.py $O/r03_08_pmcA_m3 $O/r03_08_pmcB_m3 $O/r03_08_pmcC_m3 > $O/r03_08_pmc_quad.md 2>&1; head -30 $O/r03_08_pmc_quad.md
python tools/pmc_summary.py $O/r03_08_pmcA_m0 $O/r03_08_pmcB_m0 $O/r03_08_pmcC_m0 > $O/r03_08_pmc_old.md 2>&1; head -30 $O/r03_08_pmc_old.md
timeout -k 10 300 python -u bench.py --steps 10 --warmup 4 > $O/r03_08_bench.log 2>&1 || { tail -30 $O/r03_08_bench.log; exit 1; }
grep '"metric"' $O/r03_08_bench.log | cut -c1-1500
