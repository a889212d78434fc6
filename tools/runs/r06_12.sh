#!/bin/bash
# r06 pass 12: HBM stream-rate probes (copy / add / fill; vectors in flight, grid, nontemporal).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_12; mkdir -p $O
cd $R
timeout -k 10 400 python -u tools/diag/hbm_copy.py --so /tmp/hbm_copy.so > $O/hbm.jsonl 2> $O/hbm.err || { tail -20 $O/hbm.err; exit 1; }
cat $O/hbm.jsonl
