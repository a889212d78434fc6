#!/bin/bash
# Round 4, GPU pass 28: same-box A/B of conv3x3p before (gpurun_alt/: the committed kernel) and
# after (asm epilogue image accesses, EP 2's z a tile ahead): isolated kernels and full steps,
# alternating.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04_28}; mkdir -p $O
cd $R
python3 -c "import sys; sys.path.insert(0, 'gpurun_alt'); import consensusml_amd; print(consensusml_amd.__file__)"
for i in 1 2; do
  timeout -k 10 120 python -u bench/conv3x3p.py --json-out $O/p3_new.jsonl >> $O/p3.log 2>&1 || { tail -30 $O/p3.log; exit 1; }
  timeout -k 10 120 python -u gpurun_alt/bench/conv3x3p.py --json-out $O/p3_old.jsonl >> $O/p3.log 2>&1 || { tail -30 $O/p3.log; exit 1; }
done
for f in p3_new p3_old; do echo $f; cat $O/$f.jsonl | cut -c1-120; done
B="--steps 12 --warmup 4 --no-baseline --b256-batch 0 --virtual-workers 0"
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py $B --json-out $O/resnet_new_$i.json >> $O/resnet.log 2>&1 || { tail -30 $O/resnet.log; exit 1; }
  timeout -k 10 300 python -u gpurun_alt/bench.py $B --json-out $O/resnet_old_$i.json >> $O/resnet.log 2>&1 || { tail -30 $O/resnet.log; exit 1; }
done
for f in $O/resnet_*.json; do python3 -c "import json,sys; print(sys.argv[1], json.load(open(sys.argv[1]))['ms_per_step'])" $f; done
