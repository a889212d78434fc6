#!/bin/bash
# Round 2, GPU pass 11: batched SMO kernel tests + timing, RF fit timing after the device-side
# feature draws (+ kernel stats), FETCH_SIZE / WRITE_SIZE calibration at 64 MiB..4 GiB, and the
# Multi-Krum / trimmed-mean configs at 8 virtual workers with f >= 1.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r02_11_* $O/cal_f $O/cal_w $O/rf_stats
timeout -k 10 300 python -u -m pytest tests/test_svm_gpu.py tests/test_select_gpu.py tests/test_hist_trees.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/r02_11_pytest.log 2>&1 || { tail -30 $O/r02_11_pytest.log; exit 1; }
tail -1 $O/r02_11_pytest.log
timeout -k 10 300 python -u bench/svm_smo.py > $O/r02_11_svm.jsonl 2>$O/r02_11_svm.err || { tail -20 $O/r02_11_svm.err; exit 1; }
cat $O/r02_11_svm.jsonl
timeout -k 10 300 python -u bench/reference_timings.py > $O/r02_11_reftimings.jsonl 2>$O/r02_11_ref.err || { tail -20 $O/r02_11_ref.err; exit 1; }
cat $O/r02_11_reftimings.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rf_stats -o run -- python $R/bench/reference_timings.py --reps 2 > $O/r02_11_rfprof.log 2>&1 || { tail -20 $O/r02_11_rfprof.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/cal_f -o run -- python $R/tools/diag/fetch_calibration.py --manifest $O/r02_11_manifest.json > $O/r02_11_calf.log 2>&1 || { tail -20 $O/r02_11_calf.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/cal_w -o run -- python $R/tools/diag/fetch_calibration.py > $O/r02_11_calw.log 2>&1 || { tail -20 $O/r02_11_calw.log; exit 1; }
cd $R
python tools/diag/fetch_calibration_report.py $O/r02_11_manifest.json $O/cal_f $O/cal_w > $O/r02_11_calibration.md 2>&1 || true
cat $O/r02_11_calibration.md
for c in resnet_mkrum resnet_trimmed; do
timeout -k 10 400 python -u bench/configs.py --config $c --virtual-workers 8 --batch 256 --steps 10 --warmup 3 --json-out $O/r02_11_configs.jsonl > $O/r02_11_$c.log 2>&1 || { tail -20 $O/r02_11_$c.log; exit 1; }
done
cut -c1-400 $O/r02_11_configs.jsonl
