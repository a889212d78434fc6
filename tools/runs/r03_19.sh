#!/bin/bash
# Round 3, GPU pass 19: epilogue operand batches of the fused 1x1 kernels at MT = 2 (link: 8 rows,
# BN + residual: 4 rows per batch; default 4 / 2), built as altso/_C_rb.so: families + step A/B by
# swapping the extension between runs (same box).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r03_19_*
SO=consensusml_amd/_C.cpython-310-x86_64-linux-gnu.so
cp $SO /tmp/_C_default.so
fam() {  # tag
  timeout -k 10 300 python -u bench/conv1x1g.py --json-out $O/r03_19_fam_$1.jsonl > $O/r03_19_fam_$1.log 2>&1 || { tail -20 $O/r03_19_fam_$1.log; return 1; }
}
step() {  # tag
  timeout -k 10 300 python -u bench.py --steps 12 --warmup 4 --b256-batch 0 --no-baseline --virtual-workers 0 > $O/r03_19_$1.log 2>&1 || { tail -20 $O/r03_19_$1.log; return 1; }
  python -c "import json; d=json.loads([l for l in open('$O/r03_19_$1.log') if l.startswith('{\"metric')][0]); print('$1', d['ms_per_step'], d['value'])" | tee -a $O/r03_19_ab.txt
}
fam def && step def0 && cp altso/_C_rb.so $SO && fam rb && step rb0 && cp /tmp/_C_default.so $SO && step def1 && cp altso/_C_rb.so $SO && step rb1 && cp /tmp/_C_default.so $SO || exit 1
python - <<'PY'
import json
def load(t):
    return {json.loads(l)["name"]: json.loads(l) for l in open(f"gpurun_out/r03_19_fam_{t}.jsonl") if l.startswith("{") and '"name"' in l}
a, b = load("def"), load("rb")
for k in a:
    print(f"{a[k]['kind']:11s} {k:22s} default {a[k]['old_ms']:.3f}  rb {b[k]['old_ms']:.3f}")
PY
