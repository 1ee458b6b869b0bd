#!/bin/bash
# Forward-kernel variant timings (sweep_forward.py), optionally after the
# direct-path parity tests.
# Usage: scripts/gpu_log_r3.sh <outdir> ["variants"] [skip-tests]
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3k}; mkdir -p $O
cd $GRAFT_REPO_ROOT
if [ -z "$3" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_longseries.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
  rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
V="${2:-MDP_PAIR_STORE=0;MDP_PAIR_STORE=0,MDP_FAST_LOG=0;MDP_JIT=1;MDP_PAIR_STORE=0,MDP_READ_COLS=1;MDP_PAIR_STORE=0;MDP_PAIR_STORE=0,MDP_FAST_LOG=0;MDP_JIT_HACK=1}"
timeout -k 10 300 python scripts/sweep_forward.py --configs 2,3 --steps 100 --variants "$V" > $O/sweep.jsonl 2> $O/sweep.err
