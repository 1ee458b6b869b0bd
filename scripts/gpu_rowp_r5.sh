#!/bin/bash
# Round-5 A/B of the fused prologue's per-row pressures (MDP_JIT_ROWP) on
# config 2: option parity, fused-vs-Q-row bit identity with it on, a sweep
# alternating the variants, and phase stamps (diag library).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5/rowp
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_options.py -m gpu -x -q -k "ROWP" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_opt.log 2>&1 || { tail -30 $O/pytest_opt.log; exit 1; }
tail -1 $O/pytest_opt.log
MDP_JIT_ROWP=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "large_grids or file_runs or fused or random_problems" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_par.log 2>&1 || { tail -30 $O/pytest_par.log; exit 1; }
tail -1 $O/pytest_par.log
timeout -k 10 300 python scripts/sweep_forward.py --configs 2,3 --steps 50 --variants "MDP_JIT_ROWP=0;MDP_JIT_ROWP=1;MDP_JIT_ROWP=0;MDP_JIT_ROWP=1" > $O/sweep.jsonl 2>&1 || { tail $O/sweep.jsonl; exit 1; }
cat $O/sweep.jsonl
timeout -k 10 300 python scripts/sweep_forward.py --configs 2 --diag --steps 30 --variants "MDP_JIT_ROWP=0;MDP_JIT_ROWP=1" > $O/diag.txt 2>&1 || { tail $O/diag.txt; exit 1; }
grep -A1 "back to back" $O/diag.txt | grep k_forward
