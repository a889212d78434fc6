#!/bin/bash
# Round 4, GPU pass 35: the down-sample tail's BN-folded weight concat in two launches (scaled_cat):
# the fused-backward / ResNet tests first, then pass 26's full validation (GPU suite, smoke(), the
# default bench line, batch-2048 kernel profile).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_35; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_bwd_fusion_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/quick.txt 2>&1 || { tail -40 $O/quick.txt; exit 1; }
tail -1 $O/quick.txt
OUT=r04_35 bash $R/tools/runs/r04_g26.sh
