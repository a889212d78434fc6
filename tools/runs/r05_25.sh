#!/bin/bash
# r05 pass 25: multi_copy with multi-round workgroups: test + isolated throughput.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_25; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k multi_copy > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 300 python -u bench/multi_copy.py > $O/multi_copy.jsonl 2> $O/mc.err || { tail -20 $O/mc.err; exit 1; }
cat $O/multi_copy.jsonl
for rep in 1 2; do
for m in 2 3; do
CML_C1G=$m timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-baseline --b256-batch 0 --virtual-workers 0 > $O/bench_c1g${m}_${rep}.log 2>&1 || { tail -20 $O/bench_c1g${m}_${rep}.log; exit 1; }
echo "c1g=$m rep=$rep $(grep '^{' $O/bench_c1g${m}_${rep}.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done
done
cd /tmp && export TMPDIR=/tmp
CML_C1G=3 timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw -o run -- python3 $R/bench.py --steps 6 --warmup 3 --no-baseline --b256-batch 0 --virtual-workers 0 --profile-marker > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
db=$(find $O/raw -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 400 --out $O/kernels_c1g3.md
python3 $R/tools/kernel_classes.py $O/kernels_c1g3.md > $O/classes_c1g3.md || true
rm -rf $O/raw
head -2 $O/kernels_c1g3.md; head -5 $O/classes_c1g3.md
