#!/bin/bash
# Round 2, GPU pass 30: glds conv GEMM variants (tile / buffers) vs MIOpen.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -f $O/r02_30_*
for v in 2 4; do
CML_CONV_GEMM_VARIANT=$v timeout -k 10 300 python -u bench/conv3x3.py > $O/r02_30_v$v.jsonl 2>$O/r02_30.err || { tail -20 $O/r02_30.err; exit 1; }
python - $v <<'PY'
import json,sys
v=sys.argv[1]
for l in open(f"gpurun_out/r02_30_v{v}.jsonl"):
    r=json.loads(l); print("v"+v, r['C'],r['H'],'fwd lib/glds',r['miopen_ms'],r['glds_fwd_ms'],'dgrad lib/glds',r['miopen_dgrad_ms'],r['glds_dgrad_ms'],'err',round(r['glds_fwd_err'],4),round(r['glds_dgrad_err'],4))
PY
done
