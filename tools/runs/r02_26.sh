#!/bin/bash
# Round 2, GPU pass 26: 3x3 weight gradient (wgrad1x1.hip TAP) vs MIOpen.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
timeout -k 10 400 python -u bench/conv3x3.py > $O/r02_26_conv3x3.jsonl 2>$O/r02_26.err || { tail -20 $O/r02_26.err; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r02_26_conv3x3.jsonl"):
    r=json.loads(l); print(r['C'],r['H'],'wgrad lib/own/own+pro',r['miopen_wgrad_ms'],r['own_wgrad_ms'],r['own_wgrad_pro_ms'],'err',round(r['own_wgrad_err'],4),'| fwd lib/glds',r['miopen_ms'],r['glds_fwd_ms'],'dgrad lib/glds',r['miopen_dgrad_ms'],r['glds_dgrad_ms'])
PY
