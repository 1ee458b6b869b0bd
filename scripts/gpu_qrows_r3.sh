#!/bin/bash
# k_qrows phase-1 work (round 3): parity of every path that runs k_qrows,
# phase stamps and repeated timings on
# config 3, the LDS counter pass.  Output: gpurun_out/<name>/
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3q}; mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layout.py tests/test_gpu_highvar.py tests/test_gpu_longseries.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/sweep_forward.py --configs 3 --steps 50 --diag --variants "MDP_JIT=1;MDP_JIT=1" > $O/diag.txt 2> $O/diag.err || exit $?
timeout -k 10 300 python scripts/sweep_forward.py --configs 3 --steps 100 --variants "MDP_JIT=1;MDP_JIT=1;MDP_JIT=1;MDP_JIT=1" > $O/sweep.jsonl 2> $O/sweep.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 150 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --kernel-trace --output-format csv -d $O/pmc_c3 -o run -- python3 $R/bench.py --config 3 --no-cpu-baseline --steps 3 --warmup 1 > $O/pmc_c3.json 2> $O/pmc_c3.err || exit $?
echo done
