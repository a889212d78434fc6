#!/bin/bash
# Round 4, GPU pass 36: batch-256 step profile of the final code (pass 21's script).
OUT=r04_36 bash $GRAFT_REPO_ROOT/tools/runs/r04_g21.sh
