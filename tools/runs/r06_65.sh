#!/bin/bash
# r06 pass 65: final-code validation (after the plain-link dgrad) -- the full GPU test suite (as the driver runs it), smoke(),
# the default bench, and a 2-rank gloo rehearsal of the bench on one GPU.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_65; mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json
r=json.loads([l for l in open('$O/bench.json') if l.startswith('{')][0])
print({k: r.get(k) for k in ['value','ms_per_step','agg_overhead_vs_allreduce','engine_step_ms','krum_n8_virtual_samples_per_s','krum_n8_virtual_overhead','b256_ms_per_step','b256_agg_overhead_vs_allreduce','peak_mem_gib']})"
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --dist-backend gloo --batch 128 --steps 3 --warmup 1 --b256-batch 0 --virtual-workers 0 --no-baseline > $O/gloo2.log 2>&1 || { tail -30 $O/gloo2.log; exit 1; }
grep '^{' $O/gloo2.log > $O/gloo2.json
python3 -c "
import json
r=json.loads(open('$O/gloo2.json').readline())
print('gloo 2', {k: r.get(k) for k in ['value','n_gpus','world_size_seen','replicas_identical','loss_finite','dist_backend']})"
