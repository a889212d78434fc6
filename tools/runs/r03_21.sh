#!/bin/bash
# Round 3, GPU pass 21: exact-threshold random forests on the device (ExactForest: rank bins,
# in-kernel candidate sampling, level-synchronous growth) in the reference analysis; the full
# default analysis with --device cuda, wall time and parity table.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r03_21_*
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_select_gpu.py > $O/r03_21_tests.txt 2>&1 || { tail -40 $O/r03_21_tests.txt; exit 1; }
tail -2 $O/r03_21_tests.txt
mkdir -p $O/r03_21_ref
t0=$SECONDS
timeout -k 10 600 python -u -m consensusml_amd.select --rdata refdata/sesetfilt_degseahack_targetaml.rda --device cuda --out $O/r03_21_ref > $O/r03_21_ref.log 2>&1 || { tail -30 $O/r03_21_ref.log; exit 1; }
echo "reference analysis wall (incl. python start): $((SECONDS - t0)) s" | tee $O/r03_21_wall.txt
tail -5 $O/r03_21_ref.log
python -c "import json; print(json.load(open('$O/r03_21_ref/summary.json'))['stage_seconds'])"
python tools/reference_parity_report.py $O/r03_21_ref/standouttable.csv --ref refdata/standouttable.csv > $O/r03_21_parity.md 2>&1 || { tail -20 $O/r03_21_parity.md; exit 1; }
cat $O/r03_21_parity.md
