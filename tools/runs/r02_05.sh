#!/bin/bash
# Round 2, GPU pass 5: fused vs unfused bottleneck diagnostics.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/diag/fused_block_diag.py 2>&1 | grep -v amdgpu.ids
