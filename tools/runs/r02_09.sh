#!/bin/bash
# Round 2, GPU pass 9: robustness benchmark (rule x attack, n=8 virtual workers, f=2) on the GPU
# kernels for the MLP and resnet_tiny tasks, plus its GPU test.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -f $O/r02_rob_*.jsonl $O/r02_rob.md
timeout -k 10 300 python -u -m pytest tests/test_robustness.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/r02_09_pytest.log 2>&1 || { tail -30 $O/r02_09_pytest.log; exit 1; }
tail -1 $O/r02_09_pytest.log
timeout -k 10 400 python -u bench/robustness.py --task mlp --jsonl $O/r02_rob_mlp.jsonl --md $O/r02_rob.md > $O/r02_09_mlp.log 2>&1 || { tail -20 $O/r02_09_mlp.log; exit 1; }
timeout -k 10 900 python -u bench/robustness.py --task resnet_tiny --jsonl $O/r02_rob_resnet_tiny.jsonl --md $O/r02_rob.md > $O/r02_09_rn.log 2>&1 || { tail -20 $O/r02_09_rn.log; exit 1; }
cat $O/r02_rob.md
