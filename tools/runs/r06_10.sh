#!/bin/bash
# r06 pass 10: batch-2560 kernel table + classes; the full default bench (every block).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_10; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw -o run -- python3 $R/bench.py --steps 6 --warmup 3 --no-baseline --b256-batch 0 --virtual-workers 0 --profile-marker > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
db=$(find $O/raw -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 400 --out $O/kernels_b2560.md > /dev/null
rm -rf $O/raw
python3 $R/tools/kernel_classes.py $O/kernels_b2560.md > $O/classes_b2560.md
head -3 $O/kernels_b2560.md
cat $O/classes_b2560.md
cd $R
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json
r=json.loads([l for l in open('$O/bench.json') if l.startswith('{')][0])
print({k: r.get(k) for k in ['value','ms_per_step','agg_overhead_vs_allreduce','engine_step_ms','krum_n8_virtual_samples_per_s','krum_n8_virtual_overhead','b256_ms_per_step','b256_agg_overhead_vs_allreduce','peak_mem_gib']})"
