#!/bin/bash
# GPU pass 28: full GPU test suite, smoke(), BERT steady-state profile with the MFMA attention.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu28.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu28.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke28.log 2>&1; rc=$?
tail -2 gpurun_out/smoke28.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/raw28 -o run -- python3 $R/bench/configs.py --config bert_geomed --virtual-workers 8 --batch 32 --steps 4 --warmup 2 --profile-marker > $R/gpurun_out/prof28_bert.log 2>&1 || exit $?
db=$(find $R/gpurun_out/raw28 -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 4 --top 45 --out $R/gpurun_out/prof28_bert_kernels.md
rm -rf $R/gpurun_out/raw28
