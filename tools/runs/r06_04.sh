#!/bin/bash
# r06 pass 4: GPU tests of this round's changes (gemm_w4, flash attention at S 4096 / 8192, the
# weights guard state, ordered Grams at one rank, overlapped delayed-gossip mix); Llama-3-8B
# loopback gossip step with the exp and the ring graph + kernel table; rocprofv3 --pmc passes
# over the hot kernels (tools/diag/pmc_targets.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_04; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm_w4_gpu.py tests/test_flash_attn_gpu.py tests/test_weights_guard.py tests/test_gram_precision_gpu.py tests/test_engine_gpu.py tests/test_loopback.py tests/test_dist_gpu.py tests/test_direct_grads_gpu.py tests/test_gossip_graphs.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for g in exp ring; do
  timeout -k 10 600 python -u bench/configs.py --config llama_gossip --loopback --gossip-graph $g --steps 4 --warmup 2 --no-baseline --json-out $O/llama_$g.jsonl > $O/llama_$g.log 2>&1 || { tail -30 $O/llama_$g.log; exit 1; }
  echo "llama $g"; cut -c1-400 $O/llama_$g.jsonl
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace -d $O/rawl -o run -- python3 $R/bench/configs.py --config llama_gossip --loopback --steps 3 --warmup 2 --no-baseline --profile-marker > $O/prof_llama.log 2>&1 || { tail -20 $O/prof_llama.log; exit 1; }
db=$(find $O/rawl -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 3 --top 60 --out $O/llama_kernels.md
rm -rf $O/rawl
head -24 $O/llama_kernels.md | cut -c1-200
echo "pmc passes"
i=0
for grp in "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE" "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 400 rocprofv3 --output-format csv --pmc $grp -d $O/pmc$i -o run -- python3 $R/tools/diag/pmc_targets.py > $O/pmc$i.log 2>&1 || { echo "pmc$i failed"; tail -10 $O/pmc$i.log; exit 1; }
  echo "pmc$i done"
  f=$(find $O/pmc$i -name '*counter_collection.csv' -print -quit); mv "$f" $O/pmc$i/run_counter_collection.csv
  find $O/pmc$i -mindepth 1 -not -name run_counter_collection.csv -delete 2>/dev/null || true
done
python3 $R/tools/pmc_summary.py $O/pmc1 $O/pmc2 $O/pmc3 > $O/pmc_targets.md
head -40 $O/pmc_targets.md | cut -c1-250
