#!/bin/bash
# r05 pass 48: full GPU suite + smoke + bench (checkpoint after the stride-2 tall tile).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_48; mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -3 $O/gputests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log > $O/bench.json
python3 -c "import json; d=json.load(open('$O/bench.json')); print({k: d[k] for k in ('value','ms_per_step','agg_overhead_vs_allreduce','b256_ms_per_step','b256_agg_overhead_vs_allreduce','b256_engine_step_ms','early_grams_per_step') if k in d})"

