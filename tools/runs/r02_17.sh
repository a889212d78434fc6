#!/bin/bash
# Round 2, GPU pass 17: BN kernel bandwidth + FETCH_SIZE calibration below the split-launch size.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r02_17_* $O/cal_f $O/cal_w
timeout -k 10 300 python -u bench/bn_kernels.py > $O/r02_17_bn.jsonl 2>$O/r02_17_bn.err || { tail -20 $O/r02_17_bn.err; exit 1; }
cat $O/r02_17_bn.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --output-format csv --pmc FETCH_SIZE -d $O/cal_f -o run -- python $R/tools/diag/fetch_calibration.py --manifest $O/r02_17_manifest.json > $O/r02_17_calf.log 2>&1 || { tail -20 $O/r02_17_calf.log; exit 1; }
timeout -s KILL 120 rocprofv3 --output-format csv --pmc WRITE_SIZE -d $O/cal_w -o run -- python $R/tools/diag/fetch_calibration.py > $O/r02_17_calw.log 2>&1 || { tail -20 $O/r02_17_calw.log; exit 1; }
cd $R
find $O/cal_f $O/cal_w -name "*.csv" ! -name "*counter_collection.csv" -delete
python tools/diag/fetch_calibration_report.py $O/r02_17_manifest.json $O/cal_f $O/cal_w > $O/r02_17_calibration.md
cat $O/r02_17_calibration.md
