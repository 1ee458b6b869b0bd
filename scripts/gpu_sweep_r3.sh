set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3c; mkdir -p $O
timeout -k 10 300 python scripts/sweep_forward.py --configs 2,3 --steps 50 --variants "MDP_JIT=1;MDP_FUSED=0;MDP_FUSED=0,MDP_QROWS_XCD=0;MDP_FUSED=1,MDP_EPL=1;MDP_FUSED_COLS=1" > $O/sweep.jsonl 2> $O/sweep.err && \
timeout -k 10 300 python scripts/sweep_forward.py --configs 2,3 --steps 20 --diag --variants "MDP_JIT=1" > $O/diag.txt 2>> $O/sweep.err
