#!/bin/bash
# Forward kernels with DPP-broadcast Q chunks (MDP_JIT_DPPQ=<mode>, arg 2): parity of
# every forward path against the oracle with the knob on, then alternating
# timings against the default on configs 2, 3 and 6.  Output: gpurun_out/<name>/
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3dq}; mkdir -p $O
cd $GRAFT_REPO_ROOT
MDP_JIT_DPPQ=${2:-1} timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layout.py tests/test_gpu_longseries.py tests/test_gpu_highvar.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/sweep_forward.py --configs 2,3,6 --steps 50 --variants "MDP_JIT_DPPQ=0;MDP_JIT_DPPQ=${2:-1};MDP_JIT_DPPQ=0;MDP_JIT_DPPQ=${2:-1};MDP_JIT_DPPQ=0;MDP_JIT_DPPQ=${2:-1}" > $O/sweep.jsonl 2> $O/sweep.err || exit $?
echo done
