#!/bin/bash
# Round 3, GPU pass 3: conv1x1g with the prologue applied once per k-step in LDS (default) vs on
# the B fragments (CML_C1G_FRAG=1); PerfPolicy-ported fusion tests; step A/B (auto vs regstage).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r03_03_*
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 600 $T tests/test_conv1x1g_gpu.py tests/test_bwd_fusion_gpu.py tests/test_conv1x1_bn_gpu.py tests/test_kernels_gpu.py > $O/r03_03_tests.log 2>&1 || { tail -40 $O/r03_03_tests.log; exit 1; }
tail -3 $O/r03_03_tests.log
timeout -k 10 300 python -u bench/conv1x1g.py > $O/r03_03_c1g_tl.log 2>&1 || { tail -30 $O/r03_03_c1g_tl.log; exit 1; }
cat $O/r03_03_c1g_tl.log
CML_C1G_FRAG=1 timeout -k 10 300 python -u bench/conv1x1g.py > $O/r03_03_c1g_frag.log 2>&1 || { tail -30 $O/r03_03_c1g_frag.log; exit 1; }
tail -1 $O/r03_03_c1g_frag.log
timeout -k 10 300 python -u bench.py --no-baseline --virtual-workers 0 --b256-batch 0 > $O/r03_03_bench_auto.log 2>&1 || { tail -20 $O/r03_03_bench_auto.log; exit 1; }
grep '^{' $O/r03_03_bench_auto.log | cut -c1-300
CML_C1G=0 timeout -k 10 300 python -u bench.py --no-baseline --virtual-workers 0 --b256-batch 0 > $O/r03_03_bench_old.log 2>&1 || { tail -20 $O/r03_03_bench_old.log; exit 1; }
grep '^{' $O/r03_03_bench_old.log | cut -c1-300
timeout -k 10 300 $T tests/test_batched_workers_gpu.py > $O/r03_03_batched.log 2>&1 || { tail -40 $O/r03_03_batched.log; exit 1; }
tail -3 $O/r03_03_batched.log
timeout -k 10 300 python -u bench/configs.py --config bert_geomed --virtual-workers 8 --batch 32 --steps 10 --warmup 3 > $O/r03_03_bert_b.log 2>&1 || { tail -20 $O/r03_03_bert_b.log; exit 1; }
grep '^{' $O/r03_03_bert_b.log | cut -c1-600
CML_BATCHED_WORKERS=0 timeout -k 10 300 python -u bench/configs.py --config bert_geomed --virtual-workers 8 --batch 32 --steps 10 --warmup 3 > $O/r03_03_bert_s.log 2>&1 || { tail -20 $O/r03_03_bert_s.log; exit 1; }
grep '^{' $O/r03_03_bert_s.log | cut -c1-600
timeout -k 10 300 $T -s tests/test_gram_precision_gpu.py > $O/r03_03_gramprec.log 2>&1 || { tail -40 $O/r03_03_gramprec.log; exit 1; }
grep "rel distance\|passed\|failed" $O/r03_03_gramprec.log
