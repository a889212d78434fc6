#!/bin/bash
# r06 pass 31: stem / ResNet GPU tests after the layer-1.0 dgrad GEMM default; the full default
# bench (as the driver runs it: headline + b256 + virtual-worker blocks).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_31; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_stem_gpu.py tests/test_bn_gpu.py tests/test_bwd_fusion_gpu.py tests/test_conv1x1_bn_gpu.py tests/test_engine_gpu.py tests/test_convergence_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json
r=json.loads([l for l in open('$O/bench.json') if l.startswith('{')][0])
print({k: r.get(k) for k in ['value','ms_per_step','agg_overhead_vs_allreduce','engine_step_ms','krum_n8_virtual_samples_per_s','krum_n8_virtual_overhead','b256_ms_per_step','b256_agg_overhead_vs_allreduce','peak_mem_gib']})"
