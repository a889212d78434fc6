#!/bin/bash
# Round 3, GPU pass 4: batched BERT virtual workers, centered Gram precision, quad-phase conv1x1
# kernel (bit-identical tests vs conv1x1.hip, per-shape A/B), step A/B, BERT config 4 A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r03_04_*
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_batched_workers_gpu.py > $O/r03_04_batched.log 2>&1 || { tail -40 $O/r03_04_batched.log; exit 1; }
tail -3 $O/r03_04_batched.log
timeout -k 10 300 $T -s tests/test_gram_precision_gpu.py > $O/r03_04_gramprec.log 2>&1 || { tail -40 $O/r03_04_gramprec.log; exit 1; }
grep "rel distance\|passed\|failed" $O/r03_04_gramprec.log
timeout -k 10 600 $T tests/test_conv1x1g_gpu.py > $O/r03_04_c1g_tests.log 2>&1 || { tail -40 $O/r03_04_c1g_tests.log; exit 1; }
tail -3 $O/r03_04_c1g_tests.log
timeout -k 10 300 python -u bench/conv1x1g.py > $O/r03_04_c1g.log 2>&1 || { tail -30 $O/r03_04_c1g.log; exit 1; }
cat $O/r03_04_c1g.log
timeout -k 10 300 python -u bench/configs.py --config bert_geomed --virtual-workers 8 --batch 32 --steps 10 --warmup 3 > $O/r03_04_bert_b.log 2>&1 || { tail -20 $O/r03_04_bert_b.log; exit 1; }
grep '^{' $O/r03_04_bert_b.log | cut -c1-700
CML_BATCHED_WORKERS=0 timeout -k 10 300 python -u bench/configs.py --config bert_geomed --virtual-workers 8 --batch 32 --steps 10 --warmup 3 > $O/r03_04_bert_s.log 2>&1 || { tail -20 $O/r03_04_bert_s.log; exit 1; }
grep '^{' $O/r03_04_bert_s.log | cut -c1-700
timeout -k 10 400 python -u bench.py --no-baseline --virtual-workers 0 --b256-batch 0 > $O/r03_04_bench_auto.log 2>&1 || { tail -20 $O/r03_04_bench_auto.log; exit 1; }
grep '^{' $O/r03_04_bench_auto.log | cut -c1-400
CML_C1G=0 timeout -k 10 400 python -u bench.py --no-baseline --virtual-workers 0 --b256-batch 0 > $O/r03_04_bench_old.log 2>&1 || { tail -20 $O/r03_04_bench_old.log; exit 1; }
grep '^{' $O/r03_04_bench_old.log | cut -c1-400
