#!/bin/bash
# r06 pass 5: rocprofv3 --pmc over the round's hot kernels (tools/diag/pmc_targets.py: the n = 8
# consensus step on ResNet-50, flash attention at the Llama layer, gemm.hip / gemm_w4 / gemm128,
# LDS-DMA weight gradients), raw CSVs summarised on the box and deleted; Llama exp-graph step
# record (phases).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_05; mkdir -p $O
cd $R
timeout -k 10 600 python -u bench/configs.py --config llama_gossip --loopback --steps 4 --warmup 2 --no-baseline --json-out $O/llama_exp.jsonl > $O/llama_exp.log 2>&1 || { tail -30 $O/llama_exp.log; exit 1; }
python3 -c "import json; r=json.loads(open('$O/llama_exp.jsonl').readline()); print(r['ms_per_step'], r.get('phase_ms_per_step'))"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE" "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 400 rocprofv3 --output-format csv --pmc $grp -d $O/pmc$i -o run -- python3 $R/tools/diag/pmc_targets.py > $O/pmc$i.log 2>&1 || { echo "pmc$i failed"; tail -10 $O/pmc$i.log; exit 1; }
  f=$(find $O/pmc$i -name '*counter_collection.csv' -print -quit)
  mkdir -p $O/c$i && mv "$f" $O/c$i/run_counter_collection.csv && rm -rf $O/pmc$i
  echo "pmc$i done"
done
python3 $R/tools/pmc_summary.py --match 'gram_|robust_weights|agg_|fa_|gemm_nt_kernel|gemm_w4|gemm128|wgrad_dma|gossip_mix' $O/c1 $O/c2 $O/c3 > $O/pmc_targets.md
python3 $R/tools/pmc_summary.py $O/c1 $O/c2 $O/c3 > $O/pmc_all.md
rm -rf $O/c1 $O/c2 $O/c3
cat $O/pmc_targets.md | cut -c1-300
