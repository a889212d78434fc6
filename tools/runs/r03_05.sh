#!/bin/bash
# Round 3, GPU pass 5: the full reference analysis on the GPU + RF 10k parity
# test, then the 100-step convergence comparison (item 3).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r03_05_*
mkdir -p $O/r03_05_ref
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
t0=$SECONDS
timeout -k 10 900 python -u -m consensusml_amd.select --rdata refdata/sesetfilt_degseahack_targetaml.rda --device cuda --out $O/r03_05_ref > $O/r03_05_ref.log 2>&1 || { tail -30 $O/r03_05_ref.log; exit 1; }
echo "reference analysis wall (incl. python start): $((SECONDS - t0)) s" | tee $O/r03_05_wall.txt
tail -5 $O/r03_05_ref.log
python tools/reference_parity_report.py $O/r03_05_ref/standouttable.csv --ref refdata/standouttable.csv > $O/r03_05_parity.md 2>&1 || { tail -20 $O/r03_05_parity.md; exit 1; }
cat $O/r03_05_parity.md
timeout -k 10 600 $T tests/test_reference_rdata_parity.py -m gpu > $O/r03_05_rf10k.log 2>&1 || { tail -30 $O/r03_05_rf10k.log; exit 1; }
tail -3 $O/r03_05_rf10k.log
timeout -k 10 1000 python -u bench/convergence.py --steps 100 --batch 128 --out $O/r03_05_conv > $O/r03_05_conv.log 2>&1 || { tail -30 $O/r03_05_conv.log; exit 1; }
cat $O/r03_05_conv.log | tail -3
