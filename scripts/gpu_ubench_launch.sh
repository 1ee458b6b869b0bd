#!/bin/bash
# launch-overhead microbenchmark under a few runtime settings
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3f}; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 60 ./scripts/ubench/launch_overhead > $O/default.txt 2>&1 && \
ROC_SYSTEM_SCOPE_SIGNAL=0 timeout -k 10 60 ./scripts/ubench/launch_overhead > $O/sysscope0.txt 2>&1 && \
AMD_DIRECT_DISPATCH=0 timeout -k 10 60 ./scripts/ubench/launch_overhead > $O/nodirect.txt 2>&1
