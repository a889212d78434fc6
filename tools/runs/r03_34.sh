#!/bin/bash
# Round 3, GPU pass 34: passes 33 (compact layer-4 downsample A/B) and 32 (profiles, small-M A/B) in
# one call.
set -o pipefail
bash $GRAFT_REPO_ROOT/tools/runs/r03_33.sh && bash $GRAFT_REPO_ROOT/tools/runs/r03_32.sh
