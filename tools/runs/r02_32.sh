#!/bin/bash
# Round 2, GPU pass 32: 3x3 forward on conv_gemm.hip with bn2's statistics in the epilogue --
# numerics, per-layer timing vs MIOpen + bn_stats, bench A/B (CML_CONV3X3_BN_STATS).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -f $O/r02_32_*
timeout -k 10 400 python -u -m pytest tests/test_conv1x1_bn_gpu.py tests/test_bwd_fusion_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/r02_32_pytest.log 2>&1 || { tail -30 $O/r02_32_pytest.log; exit 1; }
tail -1 $O/r02_32_pytest.log
timeout -k 10 300 python -u bench/conv3x3.py > $O/r02_32_conv3x3.jsonl 2>$O/r02_32.err || { tail -20 $O/r02_32.err; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r02_32_conv3x3.jsonl"):
    r=json.loads(l); print(r['C'],r['H'],'lib fwd+stats',round(r['miopen_ms']+r['bn_stats_ms'],4),'glds fwd / fwd+stats',r['glds_fwd_ms'],r['glds_fwd_stats_ms'])
PY
for f in 0 1 0 1; do
CML_CONV3X3_BN_STATS=$f timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-baseline --virtual-workers 0 > $O/r02_32_bench$f.log 2>&1 || { tail -20 $O/r02_32_bench$f.log; exit 1; }
echo "conv3x3_bn_stats=$f $(grep -o '"ms_per_step": [0-9.]*' $O/r02_32_bench$f.log)"
done
cd /tmp && export TMPDIR=/tmp
for f in 0 1; do
CML_CONV3X3_BN_STATS=$f timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw32_$f -o run -- python3 $R/bench.py --steps 6 --warmup 2 --no-baseline --virtual-workers 0 --profile-marker > $O/r02_32_prof$f.log 2>&1 || { tail -20 $O/r02_32_prof$f.log; exit 1; }
db=$(find $O/raw32_$f -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 90 --out $O/r02_32_kernels$f.md
rm -rf $O/raw32_$f
done
