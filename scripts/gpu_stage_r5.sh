set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5/stage
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_options.py -m gpu -x -q -k "STAGE" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_opt.log 2>&1 || { tail -30 $O/pytest_opt.log; exit 1; }
tail -2 $O/pytest_opt.log
MDP_JIT_STAGE=0.3 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "large_grids or file_runs or fused" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_par.log 2>&1 || { tail -30 $O/pytest_par.log; exit 1; }
tail -2 $O/pytest_par.log
timeout -k 10 300 python scripts/sweep_forward.py --configs 2 --steps 50 --variants "MDP_JIT_STAGE=0;MDP_JIT_STAGE=0.15;MDP_JIT_STAGE=0.3;MDP_JIT_STAGE=0.45;MDP_JIT_STAGE=0.6;MDP_JIT_STAGE=0;MDP_JIT_STAGE=0.3" > $O/sweep.jsonl 2>&1 || { tail $O/sweep.jsonl; exit 1; }
cat $O/sweep.jsonl
