#!/bin/bash
# r05 pass 11: which ResNet-50 convolutions still call a library kernel (batch 2048 and 256);
# batch-2048 kernel / class tables of the current code.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_11; mkdir -p $O
cd $R
timeout -k 10 300 python tools/list_lib_convs.py 2048 > $O/lib_convs_b2048.jsonl 2> $O/lib_convs.err || { tail -20 $O/lib_convs.err; exit 1; }
cat $O/lib_convs_b2048.jsonl
timeout -k 10 300 python tools/list_lib_convs.py 256 > $O/lib_convs_b256.jsonl 2>> $O/lib_convs.err || { tail -20 $O/lib_convs.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw -o run -- python3 $R/bench.py --steps 6 --warmup 3 --no-baseline --b256-batch 0 --virtual-workers 0 --profile-marker > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
db=$(find $O/raw -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 400 --out $O/kernels_b2048.md
python3 $R/tools/kernel_classes.py $O/kernels_b2048.md > $O/classes_b2048.md || true
rm -rf $O/raw
head -4 $O/kernels_b2048.md; cat $O/classes_b2048.md
