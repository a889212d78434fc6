#!/bin/bash
# Round 2, GPU pass 42: stride-2 paths -- downsample 1x1 weight gradient on wgrad1x1.hip, stride-2
# 3x3 forward + bn2 statistics on conv_gemm.hip: numerics, then full suite, then bench A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r02_42_* $O/raw42
timeout -k 10 300 python -u -m pytest tests/test_conv1x1_bn_gpu.py -k "s2 or stride2" -x -v --timeout 120 --timeout-method thread > $O/r02_42_pytest.log 2>&1 || { tail -40 $O/r02_42_pytest.log; exit 1; }
tail -3 $O/r02_42_pytest.log
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r02_42_gputests.txt 2>&1 || { tail -40 $O/r02_42_gputests.txt; exit 1; }
tail -1 $O/r02_42_gputests.txt
for v in "CML_WGRAD1X1_S2=0 CML_CONV3X3_S2=0" "CML_WGRAD1X1_S2=1 CML_CONV3X3_S2=0" "CML_WGRAD1X1_S2=1 CML_CONV3X3_S2=1" "CML_WGRAD1X1_S2=0 CML_CONV3X3_S2=0" "CML_WGRAD1X1_S2=1 CML_CONV3X3_S2=0" "CML_WGRAD1X1_S2=1 CML_CONV3X3_S2=1"; do
tag=$(echo $v | tr -d ' =' )
env $v timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-baseline --virtual-workers 0 > $O/r02_42_bench_$tag.log 2>&1 || { tail -20 $O/r02_42_bench_$tag.log; exit 1; }
echo "$v $(grep -o '"ms_per_step": [0-9.]*' $O/r02_42_bench_$tag.log)"
done
