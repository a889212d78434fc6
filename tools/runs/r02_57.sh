#!/bin/bash
# Round 2, GPU pass 57 (= passes 55 + 56): cat-GEMM BN sums only on the 64-channel tails vs on
# every recompute tail vs off (step A/B; tails with fewer small launches), then the 2-rank gloo rehearsal of the N > 1 bench path.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r02_57_*
timeout -k 10 400 python -u -m pytest tests/test_bwd_fusion_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/r02_57_pytest.log 2>&1 || { tail -40 $O/r02_57_pytest.log; exit 1; }
tail -1 $O/r02_57_pytest.log
for cfg in "1 64" "1 256" "0 64" "1 64" "1 256" "0 64"; do
set -- $cfg
CML_CAT_BNSUMS=$1 CML_CAT_BNSUMS_MAXC=$2 timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-baseline --virtual-workers 0 > $O/r02_57_bench_$1_$2.log 2>&1 || { tail -20 $O/r02_57_bench_$1_$2.log; exit 1; }
echo "cat_bnsums=$1 maxc=$2 $(grep -o '"ms_per_step": [0-9.]*' $O/r02_57_bench_$1_$2.log)"
done
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --dist-backend gloo --batch 256 --steps 3 --warmup 1 > $O/r02_57_gloo2.log 2>&1 || { tail -30 $O/r02_57_gloo2.log; exit 1; }
grep '"metric"' $O/r02_57_gloo2.log > $O/r02_57_gloo2.json
cut -c1-3000 $O/r02_57_gloo2.json
