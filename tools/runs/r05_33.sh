#!/bin/bash
# r05 pass 33: explicit DMA waits in the flash-attention and gemm128 loops (a barrier does not wait
# for global_load_lds and hipcc inserted no wait there); conv3x3p epilogue image accesses through
# __restrict__ helpers (no compiler vmcnt(0) in front of them); one-split DMA weight gradient
# writing dW directly (Llama-3-8B linear shapes): tests, benches, step, kernel table.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_33; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_flash_attn_gpu.py tests/test_gemm_gpu.py tests/test_conv3x3p_gpu.py tests/test_bwd_fusion_gpu.py tests/test_conv3x3_layouts_gpu.py tests/test_wgrad1x1_gpu.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 300 python -u bench/flash_attn.py > $O/flash.jsonl 2> $O/flash.err || { tail -20 $O/flash.err; exit 1; }
tail -6 $O/flash.jsonl
timeout -k 10 300 python -u bench/linear_wgrad.py --llama > $O/llama_wgrad.jsonl 2> $O/llama_wgrad.err || { tail -20 $O/llama_wgrad.err; exit 1; }
cat $O/llama_wgrad.jsonl
for rep in 1 2; do
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-baseline --b256-batch 0 --virtual-workers 0 > $O/step_$rep.log 2>&1 || { tail -20 $O/step_$rep.log; exit 1; }
echo "step_$rep $(grep '^{' $O/step_$rep.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw -o run -- python3 $R/bench.py --steps 6 --warmup 3 --no-baseline --b256-batch 0 --virtual-workers 0 --profile-marker > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
db=$(find $O/raw -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 400 --out $O/kernels.md
rm -rf $O/raw
head -2 $O/kernels.md | tail -1
