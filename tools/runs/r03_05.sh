#!/bin/bash
# Round 3, GPU pass 5: the full reference analysis on the GPU, then the
# 100-step convergence comparison fused / library / Krum-8 (item 3).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r03_05_*
mkdir -p $O/r03_05_ref
t0=$SECONDS
timeout -k 10 480 python -u -m consensusml_amd.select --rdata refdata/sesetfilt_degseahack_targetaml.rda --device cuda --out $O/r03_05_ref > $O/r03_05_ref.log 2>&1 || { tail -30 $O/r03_05_ref.log; exit 1; }
echo "reference analysis wall (incl. python start): $((SECONDS - t0)) s" | tee $O/r03_05_wall.txt
tail -5 $O/r03_05_ref.log
python tools/reference_parity_report.py $O/r03_05_ref/standouttable.csv --ref refdata/standouttable.csv > $O/r03_05_parity.md 2>&1 || { tail -20 $O/r03_05_parity.md; exit 1; }
cat $O/r03_05_parity.md
timeout -k 10 600 python -u bench/convergence.py --steps 100 --batch 128 --out $O/r03_05_conv > $O/r03_05_conv.log 2>&1 || { tail -30 $O/r03_05_conv.log; exit 1; }
tail -5 $O/r03_05_conv.log
