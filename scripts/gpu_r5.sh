#!/bin/bash
# Round-5 GPU steps (gpurun), one mode per call:
#   tests  : the whole GPU suite + smoke()
#   bench  : the default bench line, and `--gpus 2 --backend gloo` (two ranks
#            bench.py starts itself, sharing the one GPU)
#   prof   : rocprofv3 kernel stats of configs 2 and 3
#   wide   : scripts/wide_timing.py on the 45 %, 60 % and 75 %-unvisited series
#   pmcw   : PMC passes of the 60 % series (k_fwd_mma)
#   diag   : phase stamps of configs 2 and 3 (libmidaspom_diag.so, `make diag`)
# Output: gpurun_out/r5/<mode>/
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5/$1
mkdir -p $O
cd $R
case "$1" in
tests)
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
  rc=$?; tail -5 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
  cat $O/smoke.log ;;
bench)
  timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench failed"; tail $O/bench_default.err; exit 1; }
  cat $O/bench_default.json
  timeout -k 10 300 python bench.py --gpus 2 --backend gloo --steps 20 --warmup 3 > $O/bench_g2_gloo.json 2> $O/bench_g2_gloo.err || { echo "bench g2 failed"; tail $O/bench_g2_gloo.err; exit 1; }
  cat $O/bench_g2_gloo.json ;;
prof)
  cd /tmp && export TMPDIR=/tmp
  for spec in "2:--steps 50 --warmup 5" "3:--steps 20 --warmup 3"; do
    CFG=${spec%%:*}; ARGS=${spec#*:}
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cfg$CFG -o run -- python3 $R/bench.py --config $CFG $ARGS --no-cpu-baseline > $O/prof_bench_cfg$CFG.json 2> $O/prof_bench_cfg$CFG.err || { echo "prof cfg$CFG failed"; tail $O/prof_bench_cfg$CFG.err; exit 1; }
    echo "prof cfg$CFG ok"
  done ;;
widetest)
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_highvar.py tests/test_gpu_options.py tests/test_gpu_layout.py -m gpu -x -q -k "wide or WIDE or structural" --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest_wide.log 2>&1
  rc=$?; tail -3 $O/pytest_wide.log; [ $rc -eq 0 ] || exit $rc ;;
wide)
  WIDE_PATHS=wide WIDE60_PATHS=default,wideplain WIDE75_PATHS=default,wideplain timeout -k 10 500 python scripts/wide_timing.py > $O/wide_timing.jsonl 2> $O/wide_timing.err || { echo "wide timing failed"; tail $O/wide_timing.err; exit 1; }
  cat $O/wide_timing.jsonl ;;
pmcw)
  bash scripts/gpu_pmc_wide.sh r5/pmcw "" default ;;
diag)
  timeout -k 10 300 python scripts/sweep_forward.py --configs 2,3 --diag --variants "MDP_JIT=1" --steps 30 > $O/diag.txt 2>&1 || { echo "diag failed"; tail $O/diag.txt; exit 1; }
  cat $O/diag.txt ;;
*) echo "mode?"; exit 2 ;;
esac
