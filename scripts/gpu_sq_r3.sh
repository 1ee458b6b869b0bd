#!/bin/bash
# Scalar-Q forward kernels (MDP_JIT_SQ=1): the direct-path parity tests with
# the knob set, then the forward timings with and without it.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3q}; mkdir -p $O
cd $GRAFT_REPO_ROOT
MDP_JIT_SQ=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_longseries.py tests/test_gpu_highvar.py -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/sweep_forward.py --configs 2,3,6 --steps 50 --variants "${2:-MDP_JIT=1;MDP_JIT_SQ=1;MDP_FUSED=0;MDP_FUSED=0,MDP_JIT_SQ=1}" > $O/sweep.jsonl 2> $O/sweep.err || exit $?
MDP_JIT_SQ=1 timeout -k 10 600 python -u scripts/wide_timing.py > $O/wide_timing.jsonl 2> $O/wide_timing.err
