#!/bin/bash
# Round 2, GPU pass 12: FETCH_SIZE / WRITE_SIZE calibration (64 MiB..4 GiB), RF fit kernel stats,
# and the robust-rule configs (full JSON lines). Large trace files are removed on the box.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r02_12_* $O/cal_f $O/cal_w $O/rf_stats
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --output-format csv --pmc FETCH_SIZE -d $O/cal_f -o run -- python $R/tools/diag/fetch_calibration.py --manifest $O/r02_12_manifest.json > $O/r02_12_calf.log 2>&1 || { tail -20 $O/r02_12_calf.log; exit 1; }
timeout -s KILL 120 rocprofv3 --output-format csv --pmc WRITE_SIZE -d $O/cal_w -o run -- python $R/tools/diag/fetch_calibration.py > $O/r02_12_calw.log 2>&1 || { tail -20 $O/r02_12_calw.log; exit 1; }
timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --stats -d $O/rf_stats -o run -- python $R/bench/reference_timings.py --reps 2 > $O/r02_12_rfprof.log 2>&1 || { tail -20 $O/r02_12_rfprof.log; exit 1; }
find $O/rf_stats -name '*kernel_trace.csv' -delete
cd $R
python tools/diag/fetch_calibration_report.py $O/r02_12_manifest.json $O/cal_f $O/cal_w > $O/r02_12_calibration.md 2>&1 || true
cat $O/r02_12_calibration.md
find $O/rf_stats -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} $O/r02_12_rf_kernel_stats.csv
head -25 $O/r02_12_rf_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
for c in resnet_mkrum resnet_trimmed; do
timeout -k 10 400 python -u bench/configs.py --config $c --virtual-workers 8 --batch 256 --steps 10 --warmup 3 --json-out $O/r02_12_configs.jsonl > $O/r02_12_$c.log 2>&1 || { tail -20 $O/r02_12_$c.log; exit 1; }
done
find $O/cal_f $O/cal_w -name "*.csv" ! -name "*counter_collection.csv" -delete
du -sh $O
