#!/bin/bash
# Round 4, GPU pass 29: same-box full-step A/B of conv3x3p before / after (the committed kernel's
# extension from gpurun_alt/ swapped in place between runs), alternating, with a heartbeat.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04_29}; mkdir -p $O
cd $R
SO=$(ls consensusml_amd/_C*.so)
cp $SO $O/../new_C.so.tmp && cp gpurun_alt/consensusml_amd/_C*.so $O/../old_C.so.tmp
B="--steps 12 --warmup 4 --no-baseline --b256-batch 0 --virtual-workers 0"
for i in 1 2 3; do
  for v in new old; do
    cp $O/../${v}_C.so.tmp $SO
    timeout -k 10 300 python -u bench.py $B --json-out $O/resnet_${v}_$i.json >> $O/resnet.log 2>&1 || { tail -30 $O/resnet.log; exit 1; }
    echo "$v $i $(python3 -c "import json,sys; print(json.load(open(sys.argv[1]))['ms_per_step'])" $O/resnet_${v}_$i.json)"
  done
done
cp $O/../new_C.so.tmp $SO
rm -f $O/../new_C.so.tmp $O/../old_C.so.tmp
