#!/bin/bash
# Phase stamps of the config-2/3 forward kernels (after idle and back to back)
# and the dispatch-ramp microbenchmark.  Output: gpurun_out/<name>/
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3d}; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 120 ./scripts/ubench/dispatch_ramp > $O/ramp.txt 2>&1 && \
timeout -k 10 300 python scripts/sweep_forward.py --configs 2,3 --steps 20 --diag --variants "${2:-MDP_JIT=1}" > $O/diag.txt 2> $O/diag.err
