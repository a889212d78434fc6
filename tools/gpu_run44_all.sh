set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_stem_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest44.log 2>&1; rc=$?; tail -3 gpurun_out/pytest44.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_run44.sh
