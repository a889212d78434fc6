#!/bin/bash
# Round 3, GPU pass 11: cat operand loads unconditional (source picked by address; pass 10: hipcc
# branched per row and waited vmcnt(0) before re-targeting in-flight loads). Cat tests, families,
# default bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r03_10_*
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bwd_fusion_gpu.py tests/test_conv1x1g_gpu.py > $O/r03_10_tests.txt 2>&1 || { tail -40 $O/r03_10_tests.txt; exit 1; }
tail -2 $O/r03_10_tests.txt
timeout -k 10 300 python -u bench/conv1x1g.py --json-out $O/r03_10_families.jsonl > $O/r03_10_families.log 2>&1 || { tail -30 $O/r03_10_families.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r03_10_families.jsonl"):
    if l.startswith("{") and "name" in l:
        d = json.loads(l); print(f"{d['kind']:11s} {d['name']:22s} old {d['old_ms']:.3f} glds {d['glds_ms']:.3f} quad {d['quad_ms']:.3f} blt {d['hipblaslt_mm_ms']:.3f}")
PY
timeout -k 10 300 python -u bench.py --steps 10 --warmup 4 > $O/r03_10_bench.log 2>&1 || { tail -30 $O/r03_10_bench.log; exit 1; }
grep '"metric"' $O/r03_10_bench.log | cut -c1-400
