#!/bin/bash
# Round 2, GPU pass 22: 3x3 data gradient as the TAP forward of rotated weights vs MIOpen dgrad.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
timeout -k 10 400 python -u bench/conv3x3.py > $O/r02_22_conv3x3.jsonl 2>$O/r02_22.err || { tail -20 $O/r02_22.err; exit 1; }
cat $O/r02_22_conv3x3.jsonl
