#!/bin/bash
# The whole GPU suite and smoke (the first half of scripts/gpu_round3.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3ck}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
