#!/bin/bash
# r06 pass 24: stride-2 1x1 (downsample) weight gradient on the stride-2 DMA kernel (one tap):
# tests, the library-conv list of a batch-2560 step, library vs own per shape, ResNet A/B
# (CML_WGRAD1X1_S2) and the 128-channel stride-2 3x3 on the own kernel (CML_WGRAD3X3_S2_MIN_CI=128).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_24; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_wgrad3x3s2_gpu.py tests/test_flash_attn_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/list_lib_convs.py 2560 > $O/lib_convs.jsonl 2> $O/lib_convs.err || { tail -20 $O/lib_convs.err; exit 1; }
cat $O/lib_convs.jsonl | cut -c1-250
timeout -k 10 300 python -u bench/wgrad_lib.py 2560 > $O/wgrad_lib.jsonl 2> $O/wgrad_lib.err || { tail -20 $O/wgrad_lib.err; exit 1; }
cat $O/wgrad_lib.jsonl | cut -c1-250
for c in 1 0 1 0; do
  CML_WGRAD1X1_S2=$c timeout -k 10 500 python -u bench.py --steps 10 --warmup 5 --no-baseline --b256-batch 0 --virtual-workers 0 > $O/b_$c.json 2> $O/b_$c.err || { tail -20 $O/b_$c.err; exit 1; }
  python3 -c "
import json
r=json.loads([l for l in open('$O/b_$c.json') if l.startswith('{')][0])
print('resnet s2 own $c', r['value'], r['ms_per_step'])"
done
for c in 128 256 128 256; do
  CML_WGRAD3X3_S2_MIN_CI=$c timeout -k 10 500 python -u bench.py --steps 10 --warmup 5 --no-baseline --b256-batch 0 --virtual-workers 0 > $O/c_$c.json 2> $O/c_$c.err || { tail -20 $O/c_$c.err; exit 1; }
  python3 -c "
import json
r=json.loads([l for l in open('$O/c_$c.json') if l.startswith('{')][0])
print('resnet 3x3s2 min_ci $c', r['value'], r['ms_per_step'])"
done
# flash attention: 8-wave (256-query) forward / dQ workgroups vs 4-wave (CML_FA_WAVES)
CML_FA_WAVES=8 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_flash_attn_gpu.py > $O/fa_tests.log 2>&1 || { tail -30 $O/fa_tests.log; exit 1; }
tail -1 $O/fa_tests.log
for wv in 4 8 4 8; do
  CML_FA_WAVES=$wv timeout -k 10 200 python -u bench/flash_attn.py --impl flash --rounds 3 > $O/fa_$wv.jsonl 2> $O/fa_$wv.err || { tail -20 $O/fa_$wv.err; exit 1; }
  echo "waves $wv"; cat $O/fa_$wv.jsonl | tail -2 | cut -c1-200
done
