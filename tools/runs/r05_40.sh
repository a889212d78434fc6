#!/bin/bash
# r05 pass 40: stride-2 3x3 data gradient (parity classes) on 128 x 128 tiles (2 workgroups / CU)
# vs 256-row tiles: step A/B and kernel tables.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_40; mkdir -p $O
cd $R
CML_CONV_GEMM_PAR128=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv3x3_s2_gpu.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
run() {   # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-baseline --b256-batch 0 --virtual-workers 0 > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  echo "$tag $(grep '^{' $O/$tag.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
}
for rep in 1 2; do
run p128_$rep CML_CONV_GEMM_PAR128=1
run base_$rep CML_CONV_GEMM_PAR128=0
done
cd /tmp && export TMPDIR=/tmp
for m in 0 1; do
CML_CONV_GEMM_PAR128=$m timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw$m -o run -- python3 $R/bench.py --steps 6 --warmup 3 --no-baseline --b256-batch 0 --virtual-workers 0 --profile-marker > $O/prof$m.log 2>&1 || { tail -20 $O/prof$m.log; exit 1; }
db=$(find $O/raw$m -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 400 --out $O/kernels_p$m.md > /dev/null
rm -rf $O/raw$m
head -2 $O/kernels_p$m.md | tail -1
grep -E "conv_gemm_kernel<.*true>" $O/kernels_p$m.md | cut -c1-200
done
