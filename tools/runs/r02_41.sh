#!/bin/bash
# Round 2, GPU pass 41: which library ops are left in the batch-2048 step (torch.profiler shapes),
# and the 1x1 weight-gradient shape set A/B (CML_WGRAD1X1_SET core / all).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r02_41_*
timeout -k 10 400 python -u tools/torch_prof_fills.py --batch 2048 --keys "aten::mm,aten::addmm,aten::convolution_backward,aten::miopen_convolution,aten::convolution,aten::_convolution" > $O/r02_41_libops.txt 2>&1 || { tail -20 $O/r02_41_libops.txt; exit 1; }
grep -A60 "=== ops containing" $O/r02_41_libops.txt | cut -c1-300 | head -60
for s in core all core all; do
CML_WGRAD1X1_SET=$s timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-baseline --virtual-workers 0 > $O/r02_41_bench_$s.log 2>&1 || { tail -20 $O/r02_41_bench_$s.log; exit 1; }
echo "wgrad1x1_set=$s $(grep -o '"ms_per_step": [0-9.]*' $O/r02_41_bench_$s.log)"
done
