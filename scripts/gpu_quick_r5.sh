#!/bin/bash
# Round-5 quick check of a forward-kernel change: fused / Q-row parity subset,
# configs 2-3 timings (three repeats) and config-2 phase stamps.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5/quick
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_options.py -m gpu -x -q -k "large_grids or file_runs or fused or random_problems or FUSED or anchor" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_par.log 2>&1 || { tail -30 $O/pytest_par.log; exit 1; }
tail -1 $O/pytest_par.log
timeout -k 10 300 python scripts/sweep_forward.py --configs 2,3 --steps 50 --variants "MDP_JIT=1;MDP_JIT=1;MDP_JIT=1" > $O/sweep.jsonl 2>&1 || { tail $O/sweep.jsonl; exit 1; }
grep -o '"config": [0-9]*\|"k_[a-z]*": [0-9.]*\|"step_us": [0-9.]*' $O/sweep.jsonl | paste -sd' ' | sed 's/"config"/\n"config"/g'
echo
timeout -k 10 300 python scripts/sweep_forward.py --configs 2 --diag --steps 20 --variants "MDP_JIT=1" > $O/diag.txt 2>&1 || { tail $O/diag.txt; exit 1; }
grep -A1 "back to back" $O/diag.txt | grep k_forward
