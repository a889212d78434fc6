#!/bin/bash
# r05 pass 47: stride-2 3x3 forwards (+ BN statistics) on gemm.hip's conv schedule (tall tile for
# 128 channels, square for 256 / 512): tests, step A/B (CML_GEMM2_S2=0 keeps conv_gemm.hip), table.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_47; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_gemm2_gpu.py tests/test_conv3x3_s2_gpu.py tests/test_bwd_fusion_gpu.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
run() {   # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-baseline --b256-batch 0 --virtual-workers 0 > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  echo "$tag $(grep '^{' $O/$tag.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
}
for rep in 1 2 3; do
run s2_$rep CML_GEMM2_S2=1
run base_$rep CML_GEMM2_S2=0
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw -o run -- python3 $R/bench.py --steps 6 --warmup 3 --no-baseline --b256-batch 0 --virtual-workers 0 --profile-marker > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
db=$(find $O/raw -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 400 --out $O/kernels.md > /dev/null
rm -rf $O/raw
head -2 $O/kernels.md | tail -1
grep -E "gemm_nt_kernel<.*true|conv_gemm_kernel" $O/kernels.md | cut -c1-200
