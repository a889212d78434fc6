#!/bin/bash
# r05 pass 9: deferred multi-bucket Gram reduce: bitwise test + engine / loopback tests, headline
# bench (b256 Krum overhead).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_09; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_weights_guard.py tests/test_loopback.py tests/test_engine_gpu.py tests/test_dist_gpu.py tests/test_gram_precision_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json
r=json.loads([l for l in open('$O/bench.json') if l.startswith('{')][0])
print({k: r.get(k) for k in ['value','ms_per_step','agg_overhead_vs_allreduce','engine_step_ms','krum_n8_virtual_overhead','b256_ms_per_step','b256_allreduce_ms_per_step','b256_agg_overhead_vs_allreduce','b256_engine_step_ms','b256_allreduce_engine_step_ms','b256_config']})"
