#!/bin/bash
# Round 2, GPU pass 10: fused flat-buffer optimizers (tests + step-time bench vs torch.optim),
# robustness table for resnet_tiny at noise 6, headline bench at the conventional batch 256/GPU.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -f $O/r02_10_*
timeout -k 10 300 python -u -m pytest tests/test_optim.py tests/test_robustness.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/r02_10_pytest.log 2>&1 || { tail -30 $O/r02_10_pytest.log; exit 1; }
tail -1 $O/r02_10_pytest.log
for m in "resnet50 fp32" "resnet50 bf16" "bert_base bf16"; do set -- $m
timeout -k 10 300 python -u bench/optim_step.py --model $1 --dtype $2 >> $O/r02_10_optim.jsonl 2>$O/r02_10_optim.err || { tail -20 $O/r02_10_optim.err; exit 1; }
done
cat $O/r02_10_optim.jsonl
timeout -k 10 600 python -u bench.py --batch 256 --steps 30 --warmup 10 > $O/r02_10_bench256.log 2>&1 || { tail -20 $O/r02_10_bench256.log; exit 1; }
grep '"metric"' $O/r02_10_bench256.log | cut -c1-1500
timeout -k 10 900 python -u bench/robustness.py --task resnet_tiny --jsonl $O/r02_10_rob_resnet_tiny.jsonl --md $O/r02_10_rob.md > $O/r02_10_rn.log 2>&1 || { tail -20 $O/r02_10_rn.log; exit 1; }
cat $O/r02_10_rob.md
