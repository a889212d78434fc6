#!/bin/bash
# r05 pass 28: ResNet headline + engine tests with direct gradients on (default).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_28; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py tests/test_dist_gpu.py tests/test_agg_multi_gpu.py tests/test_gram_precision_gpu.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log > $O/bench.json
python3 -c "import json; d=json.load(open('$O/bench.json')); print({k: d[k] for k in ('value','ms_per_step','agg_overhead_vs_allreduce','b256_ms_per_step','b256_agg_overhead_vs_allreduce','b256_engine_step_ms') if k in d})"
