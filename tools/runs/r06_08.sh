#!/bin/bash
# r06 pass 8: which ResNet-50 convolutions still run MIOpen at per-GPU batch 2560, then an
# exhaustive MIOpen search (SEARCH_DB_UPDATE) of those shapes at 2560, seeded with the shipped db.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_08; mkdir -p $O
cd $R
timeout -k 10 400 python -u tools/list_lib_convs.py 2560 > $O/lib_convs_b2560.jsonl 2> $O/lib_convs.err || { tail -20 $O/lib_convs.err; exit 1; }
cat $O/lib_convs_b2560.jsonl | cut -c1-250
