#!/bin/bash
# Round 4, GPU pass 18: conv3x3p.hip (counted LDS waits in the MFMA loop) in isolation + tests + step A/B (bench/conv3x3p.py): the kernel, its skeleton
# without MFMAs / without the per-tile DMA, the implicit-GEMM kernel it replaced; SQ counters.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04_18}; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_conv3x3p_gpu.py tests/test_bwd_fusion_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
for d in 0 1 2 3; do
  CML_CONV3P_DBG=$d timeout -k 10 120 python -u bench/conv3x3p.py --json-out $O/p3.jsonl >> $O/p3.log 2>&1 || { tail -30 $O/p3.log; exit 1; }
done
CML_CONV3P=0 timeout -k 10 120 python -u bench/conv3x3p.py --json-out $O/p3.jsonl >> $O/p3.log 2>&1 || { tail -30 $O/p3.log; exit 1; }
cat $O/p3.jsonl
B="--steps 12 --warmup 4 --no-baseline --b256-batch 0 --virtual-workers 0"
i=0
for v in 1 0 1 0; do
  i=$((i+1))
  CML_CONV3P=$v timeout -k 10 300 python -u bench.py $B --json-out $O/resnet_p3_${v}_$i.json >> $O/resnet.log 2>&1 || { tail -30 $O/resnet.log; exit 1; }
done
for f in $O/resnet_p3_*.json; do python3 -c "import json,sys; print(sys.argv[1], json.load(open(sys.argv[1]))['ms_per_step'])" $f; done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --output-format csv --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS -d $O/pmc1 -o run -- python3 $R/bench/conv3x3p.py --reps 3 > $O/pmc1.log 2>&1 || { tail -20 $O/pmc1.log; exit 1; }
python3 - $O/pmc1/run_counter_collection.csv <<'PY' > $O/pmc1.md
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in rows:
    if "conv3x3p" not in r["Kernel_Name"]:
        continue
    k = r["Kernel_Name"][:60]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    if r["Counter_Name"] == "SQ_WAVE_CYCLES":
        n[k] += 1
for k, d in agg.items():
    print(k, n[k], {c: round(v / max(n[k], 1)) for c, v in sorted(d.items())})
PY
cat $O/pmc1.md
find $O/pmc1 -type f ! -name 'run_counter_collection.csv' -delete
