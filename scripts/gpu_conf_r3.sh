#!/bin/bash
# LDS bank-conflict work (round 3): parity of the forward variants, phase
# stamps of configs 2/3, and the LDS counter pass on both.  Output:
# gpurun_out/<name>/
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3c}; mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layout.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/sweep_forward.py --configs 2,3 --steps 50 --diag --variants "MDP_JIT=1;MDP_JIT=1" > $O/diag.txt 2> $O/diag.err || exit $?
timeout -k 10 300 python scripts/sweep_forward.py --configs 2,3 --steps 100 --variants "MDP_JIT=1;MDP_JIT=1;MDP_JIT=1" > $O/sweep.jsonl 2> $O/sweep.err || exit $?
cd /tmp && export TMPDIR=/tmp
for CFG in 2 3; do
  timeout -k 10 150 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --kernel-trace --output-format csv -d $O/pmc_c$CFG -o run -- python3 $R/bench.py --config $CFG --no-cpu-baseline --steps 3 --warmup 1 > $O/pmc_c$CFG.json 2> $O/pmc_c$CFG.err || exit $?
  timeout -k 10 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY --kernel-trace --output-format csv -d $O/pmcw_c$CFG -o run -- python3 $R/bench.py --config $CFG --no-cpu-baseline --steps 3 --warmup 1 > $O/pmcw_c$CFG.json 2> $O/pmcw_c$CFG.err || exit $?
done
echo done
