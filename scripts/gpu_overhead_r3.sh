#!/bin/bash
# the forward kernel's output stores and log: measurement-only variants
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3j}; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python scripts/sweep_forward.py --configs 2,3 --steps 100 --variants "MDP_JIT=1;MDP_PAIR_STORE=0;MDP_JIT_HACK=1;MDP_JIT_HACK=2;MDP_JIT=1;MDP_PAIR_STORE=0;MDP_JIT_HACK=2;MDP_JIT_HACK=1" > $O/sweep.jsonl 2> $O/sweep.err
