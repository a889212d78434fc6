#!/bin/bash
# r06 pass 19: rocprofv3 --pmc on the stem weight gradient (gather form, batch 2560): where its
# cycles go (VALU vs MFMA vs LDS vs waits), parity-class staging on and off.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_19; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE GRBM_GUI_ACTIVE" "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --output-format csv --pmc $grp -d $O/pmc$i -o run -- python3 $R/tools/diag/pmc_targets.py --only stem --steps 3 > $O/pmc$i.log 2>&1 || { echo "pmc$i failed"; tail -10 $O/pmc$i.log; exit 1; }
  f=$(find $O/pmc$i -name '*counter_collection.csv' -print -quit)
  mkdir -p $O/c$i && mv "$f" $O/c$i/run_counter_collection.csv && rm -rf $O/pmc$i
  echo "pmc$i done"
done
python3 $R/tools/pmc_summary.py --match 'stem_' $O/c1 $O/c2 $O/c3 > $O/pmc_stem.md
rm -rf $O/c1 $O/c2 $O/c3
cat $O/pmc_stem.md | cut -c1-400
