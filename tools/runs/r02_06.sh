#!/bin/bash
# Round 2, GPU pass 6: whole-model fused / unfused vs fp32 gradient cosine.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/diag/fused_block_diag.py model 2>&1 | grep -v amdgpu.ids
