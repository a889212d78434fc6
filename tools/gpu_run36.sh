#!/bin/bash
# GPU pass 36: A/B of MIOpen's asm GTC backward-data solver (needs workspace + aux kernels) vs its
# CK alternative from the same find-db.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-baseline > gpurun_out/bench36_a.log 2>&1 || exit $?
echo "default $(tail -1 gpurun_out/bench36_a.log | cut -c90-170)"
MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-baseline > gpurun_out/bench36_b.log 2>&1 || exit $?
echo "no-gtc-bwd $(tail -1 gpurun_out/bench36_b.log | cut -c90-170) $(grep 'warmup [0-9]' gpurun_out/bench36_b.log)"
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-baseline > gpurun_out/bench36_c.log 2>&1 || exit $?
echo "default $(tail -1 gpurun_out/bench36_c.log | cut -c90-170)"
