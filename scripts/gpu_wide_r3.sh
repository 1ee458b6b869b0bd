#!/bin/bash
# wide-year parity tests and the wide timing cases
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3w}; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider -k "wide" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/wide_timing.py > $O/wide_timing.jsonl 2> $O/wide_timing.err
