#!/bin/bash
# k_qrows with the rows' explicit columns staged in LDS (MDP_QROWS_ZLDS=1)
# against reading them from L2 (=0, default): parity of every k_qrows path,
# phase stamps and alternating timings on configs 3 and 6.  Output:
# gpurun_out/<name>/
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3z}; mkdir -p $O
cd $GRAFT_REPO_ROOT
MDP_QROWS_ZLDS=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layout.py tests/test_gpu_highvar.py tests/test_gpu_longseries.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/sweep_forward.py --configs 3 --steps 30 --diag --variants "MDP_QROWS_ZLDS=1;MDP_QROWS_ZLDS=0" > $O/diag.txt 2> $O/diag.err || exit $?
timeout -k 10 400 python scripts/sweep_forward.py --configs 3,6 --steps 100 --variants "MDP_QROWS_ZLDS=1;MDP_QROWS_ZLDS=0;MDP_QROWS_ZLDS=1;MDP_QROWS_ZLDS=0;MDP_QROWS_ZLDS=1;MDP_QROWS_ZLDS=0" > $O/sweep.jsonl 2> $O/sweep.err || exit $?
echo done
