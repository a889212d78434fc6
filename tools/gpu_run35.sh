#!/bin/bash
# GPU pass 35: attribute fill / SetTensor kernels of the ResNet step to their ATen callers.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 400 python -u tools/torch_prof_fills.py > gpurun_out/fills35.txt 2>&1; rc=$?
grep -n "=== ops" -A 60 gpurun_out/fills35.txt | head -80 | cut -c1-200
exit $rc
