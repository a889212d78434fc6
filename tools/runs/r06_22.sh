#!/bin/bash
# r06 pass 22: stem_wgrad_pc_kernel timing ablations (CML_STEM_PC_ABL: 1 no staging compute,
# 2 no products, 4 no input-tile restage, 8 no producer global loads) at batch 2560.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_22; mkdir -p $O
cd $R
for a in 0 1 2 4 8 3 12 0; do
  CML_STEM_PC_ABL=$a timeout -k 10 200 python -u bench/stem_bwd.py --batch 2560 > $O/stem_$a.txt 2>&1 || { tail -20 $O/stem_$a.txt; exit 1; }
  echo "abl $a $(tail -1 $O/stem_$a.txt)"
done
