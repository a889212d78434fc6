#!/bin/bash
# r06 pass 47: cross-entropy mean / count in one launch and the grad_output / count divide inside
# the backward kernels: transformer / head / model tests, Llama smoke via the transformer tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_47; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  tests/test_transformer_ops_gpu.py tests/test_head_fusion_gpu.py tests/test_fin_affine_gpu.py \
  tests/test_convergence_gpu.py tests/test_engine_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
