#!/bin/bash
# Round 2, GPU pass 19: MT = 2 wave tiles in the fused 1x1 conv kernel -- numerics, per-shape A/B,
# identity-tail fusion A/B per stage, full-step A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -f $O/r02_19_*
timeout -k 10 400 python -u -m pytest tests/test_conv1x1_bn_gpu.py tests/test_bwd_fusion_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/r02_19_pytest.log 2>&1 || { tail -30 $O/r02_19_pytest.log; exit 1; }
tail -1 $O/r02_19_pytest.log
for m in 0 1; do
CML_C1_MT2=$m timeout -k 10 400 python -u bench/conv1x1_fused.py > $O/r02_19_c1_mt$m.jsonl 2>$O/r02_19_c1.err || { tail -20 $O/r02_19_c1.err; exit 1; }
done
python - <<'PY'
import json
a=[json.loads(l) for l in open("gpurun_out/r02_19_c1_mt0.jsonl")]
b=[json.loads(l) for l in open("gpurun_out/r02_19_c1_mt1.jsonl")]
for x,y in zip(a,b): print(x["name"], "lib", x["library_conv_ms"], "mt1", x["fused_ms"], "mt2", y["fused_ms"])
PY
CML_C1_MT2=1 timeout -k 10 400 python -u bench/bwd_fusion.py > $O/r02_19_bwdfusion.jsonl 2>$O/r02_19_bf.err || { tail -20 $O/r02_19_bf.err; exit 1; }
cat $O/r02_19_bwdfusion.jsonl
for m in 0 1; do
CML_C1_MT2=$m timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-baseline --virtual-workers 0 > $O/r02_19_bench$m.log 2>&1 || { tail -20 $O/r02_19_bench$m.log; exit 1; }
echo "mt2=$m $(grep -o '"ms_per_step": [0-9.]*' $O/r02_19_bench$m.log)"
done
