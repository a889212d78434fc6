#!/bin/bash
# r06 pass 44: the full GPU test suite (as the driver runs it) + smoke() + the default bench, on
# the final round-6 code.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_44; mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -4 $O/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json
r=json.loads([l for l in open('$O/bench.json') if l.startswith('{')][0])
print({k: r.get(k) for k in ['value','ms_per_step','agg_overhead_vs_allreduce','engine_step_ms','krum_n8_virtual_samples_per_s','krum_n8_virtual_overhead','b256_ms_per_step','b256_agg_overhead_vs_allreduce','peak_mem_gib']})"
