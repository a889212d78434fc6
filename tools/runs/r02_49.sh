#!/bin/bash
# Round 2, GPU pass 49: compact stride-2 gradient added at the even pixels by conv1 dgrad (CML_S2_LINK_DGRAD)
# numerics, bench A/B, profile.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r02_49_* $O/raw49
timeout -k 10 400 python -u -m pytest tests/test_bwd_fusion_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/r02_49_pytest.log 2>&1 || { tail -40 $O/r02_49_pytest.log; exit 1; }
tail -1 $O/r02_49_pytest.log
for f in 0 1 0 1; do
CML_S2_LINK_DGRAD=$f timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-baseline --virtual-workers 0 > $O/r02_49_bench$f.log 2>&1 || { tail -20 $O/r02_49_bench$f.log; exit 1; }
echo "s2_link=$f $(grep -o '"ms_per_step": [0-9.]*' $O/r02_49_bench$f.log)"
done
grep '^{' $O/r02_49_bench1.log > $O/r02_49_bench_on.json
grep '^{' $O/r02_49_bench0.log > $O/r02_49_bench_off.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw49 -o run -- python3 $R/bench.py --steps 6 --warmup 2 --no-baseline --virtual-workers 0 --profile-marker > $O/r02_49_prof.log 2>&1 || { tail -20 $O/r02_49_prof.log; exit 1; }
db=$(find $O/raw49 -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 90 --out $O/r02_49_kernels.md
rm -rf $O/raw49
python3 $R/tools/kernel_classes.py $O/r02_49_kernels.md
