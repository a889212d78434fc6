#!/bin/bash
# Round 4, GPU pass 12: stride-1 3x3 convs on gemm.hip (CML_CONV_GEMM2=1): kernel table and two
# more step A/Bs; HBM bytes per ResNet-50 step (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, one
# counter per run, batch 2048) -> the step's memory floor; Llama-3-8B gossip step + kernel profile.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04_12}; mkdir -p $O
cd $R
B="--steps 12 --warmup 4 --no-baseline --b256-batch 0 --virtual-workers 0"
i=0
for v in 0 1 0 1; do
  i=$((i+1))
  CML_CONV_GEMM2=$v timeout -k 10 300 python -u bench.py $B --json-out $O/resnet_g2_${v}_$i.json >> $O/resnet.log 2>&1 || { tail -30 $O/resnet.log; exit 1; }
done
cd /tmp && export TMPDIR=/tmp
CML_CONV_GEMM2=1 timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw -o run -- python3 $R/bench.py --steps 6 --warmup 3 --no-baseline --b256-batch 0 --virtual-workers 0 --profile-marker > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
db=$(find $O/raw -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 400 --out $O/kernels_b2048_g2.md
python3 $R/tools/kernel_classes.py $O/kernels_b2048_g2.md > $O/classes_b2048_g2.md || true
rm -rf $O/raw
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --output-format csv --pmc $c -d $O/pmc_$c -o run -- python3 $R/bench.py --steps 3 --warmup 2 --no-baseline --b256-batch 0 --virtual-workers 0 --profile-marker > $O/pmc_$c.log 2>&1 || { tail -20 $O/pmc_$c.log; exit 1; }
done
python3 $R/tools/pmc_step_bytes.py --steps 3 $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE > $O/step_bytes_b2048.md
cat $O/step_bytes_b2048.md
find $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE -type f ! -name 'run_counter_collection.csv' -delete
cd $R
timeout -k 10 600 python -u bench/configs.py --config llama_gossip --loopback --steps 5 --warmup 2 --json-out $O/llama.jsonl > $O/llama.log 2>&1 || { tail -30 $O/llama.log; exit 1; }
cut -c1-400 $O/llama.jsonl
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace -d $O/rawl -o run -- python3 $R/bench/configs.py --config llama_gossip --loopback --steps 3 --warmup 2 --profile-marker > $O/prof_llama.log 2>&1 || { tail -20 $O/prof_llama.log; exit 1; }
db=$(find $O/rawl -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 3 --top 60 --out $O/llama_kernels.md
rm -rf $O/rawl
head -30 $O/llama_kernels.md | cut -c1-200
