#!/bin/bash
# Round 4, GPU pass 32: stem input column sums (stem_cola) with independent loads per pixel, bn3's
# affine from the Gram-statistics finalize: the stem / Gram tests first, then pass 26's full
# validation (GPU suite, smoke(), the default bench line, batch-2048 kernel profile).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_32; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_stem_gpu.py tests/test_bwd_fusion_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/quick.txt 2>&1 || { tail -40 $O/quick.txt; exit 1; }
tail -1 $O/quick.txt
OUT=r04_32 bash $R/tools/runs/r04_g26.sh
