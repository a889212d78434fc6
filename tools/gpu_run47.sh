#!/bin/bash
# GPU pass 47: stem wgrad timing with and without the colA accumulation (diagnostic).
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 120 python tools/diag/stem_bench.py && CML_STEM_NOCOLA=1 timeout -k 10 120 python tools/diag/stem_bench.py
