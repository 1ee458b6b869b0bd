#!/bin/bash
# parity of the forward variants + the paired-store / two-column sweep
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3h}; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_longseries.py tests/test_gpu_highvar.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/sweep_forward.py --configs 2,3 --steps 50 --variants "MDP_JIT=1;MDP_PAIR_STORE=0;MDP_READ_COLS=1;MDP_PAIR_STORE=0,MDP_READ_COLS=1;MDP_JIT=1" > $O/sweep.jsonl 2> $O/sweep.err
