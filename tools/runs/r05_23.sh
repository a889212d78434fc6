#!/bin/bash
# r05 pass 23: multi_copy with per-workgroup entry slices: tests, b256 + b2048 bench, b256 table.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_23; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log > $O/bench.json
python3 -c "import json; d=json.load(open('$O/bench.json')); print({k: d[k] for k in ('value','ms_per_step','agg_overhead_vs_allreduce','b256_ms_per_step','b256_agg_overhead_vs_allreduce','b256_engine_step_ms') if k in d})"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw256 -o run -- python3 $R/bench.py --batch 256 --steps 10 --warmup 3 --no-baseline --b256-batch 0 --virtual-workers 0 --profile-marker > $O/prof256.log 2>&1 || { tail -20 $O/prof256.log; exit 1; }
db=$(find $O/raw256 -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 10 --top 500 --out $O/kernels_b256.md
rm -rf $O/raw256
head -3 $O/kernels_b256.md; grep multi_copy $O/kernels_b256.md | cut -c1-160
