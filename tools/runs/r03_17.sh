#!/bin/bash
# Round 3, GPU pass 17: policy re-check after the packed prologues / tail algebra (one call, default
# measured between the variants): bn2 sums in the cat epilogue up to 256 channels, fused bn3
# backward up to 256 planes, layer-4 recompute tails, layer-4 stride-2 downsample tail, glds family.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r03_17_*
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 12 --warmup 4 --b256-batch 0 --no-baseline --virtual-workers 0 > $O/r03_17_$tag.log 2>&1 || { tail -20 $O/r03_17_$tag.log; return 1; }
  python -c "import json,sys; d=json.loads([l for l in open('$O/r03_17_$tag.log') if l.startswith('{\"metric')][0]); print('$tag', d['ms_per_step'], d['value'], d['peak_mem_gib'])" | tee -a $O/r03_17_ab.txt
}
run default0 CML_NONE=1 && \
run bnsums256 CML_CAT_BNSUMS_MAXC=256 && \
run bn3bwd256 CML_FUSED_BN3_BWD_MAX_PLANES=256 && \
run default1 CML_NONE=1 && \
run rtail512 CML_RECOMPUTE_TAIL_MAX_PLANES=512 && \
run s2cin1024 CML_DOWN_TAIL_S2_MAX_CIN=1024 && \
run default2 CML_NONE=1 && \
run glds CML_C1G=1 && \
run bnsums128 CML_CAT_BNSUMS_MAXC=128 && \
run default3 CML_NONE=1
cat $O/r03_17_ab.txt
