#!/bin/bash
# The one gpurun recipe (round 6 folds the per-round scripts into it):
#   /usr/local/graft/bin/gpurun -- bash scripts/gpu.sh <mode> [tag] [args...]
# Output: gpurun_out/<tag>/<mode>/ (tag defaults to "run").  Every GPU step has
# its own time limit and the recipe stops at the first failing step.
#
# modes:
#   tests               the whole GPU suite, then smoke()
#   pytest  <tag> <sel> a GPU test subset (pytest -k expression <sel>)
#   bench   <tag> [cfg] bench.py lines (default line; cfg -> --config cfg)
#   rehearse            bench.py with 2 ranks over gloo on the one GPU, per config
#   prof    <tag> [cfgs]  rocprofv3 --kernel-trace --stats of bench configs (default "2 3")
#   pmc     <tag> <cfg>   PMC passes of one bench config (instruction mix, stalls,
#                         LDS, FP64 counts, FETCH/WRITE traffic) + summaries
#   traffic <tag> [cfgs]  FETCH_SIZE / WRITE_SIZE passes -> pmc_traffic_cfg*.json
#   wide    <tag>         scripts/wide_timing.py (paths from WIDE*_PATHS)
#   pmcw    <tag>         PMC passes over scripts/wide_timing.py (MFMA busy, waits, LDS)
#   sweep   <tag> <variants> [cfgs]  scripts/sweep_forward.py A/B, variants alternating twice
#   diag    <tag> [cfgs]  phase stamps (libmidaspom_diag.so, `make diag` first)
#   ubench  <tag> <name>  one scripts/ubench program (built here by make -C scripts/ubench)
set -o pipefail
R=$GRAFT_REPO_ROOT
MODE=$1
TAG=${2:-run}
O=$R/gpurun_out/$TAG/$MODE
mkdir -p $O
cd $R
PROF() {  # PROF <outdir> <pmc counters or ""> <limit s> -- command...
  local d=$1 pmc=$2 lim=$3
  shift 4
  if [ -n "$pmc" ]; then
    (cd /tmp && TMPDIR=/tmp timeout -k 10 $lim rocprofv3 --pmc $pmc --kernel-trace --output-format csv -d $d -o run -- "$@")
  else
    (cd /tmp && TMPDIR=/tmp timeout -k 10 $lim rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- "$@")
  fi
}
case "$MODE" in
tests)
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
  rc=$?; tail -5 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
  cat $O/smoke.log ;;
pytest)
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "$3" > $O/pytest.log 2>&1
  rc=$?; tail -5 $O/pytest.log; exit $rc ;;
bench)
  ARGS=""; [ -n "$3" ] && ARGS="--config $3"
  timeout -k 10 300 python bench.py $ARGS > $O/bench$3.json 2> $O/bench$3.err || { echo "bench failed"; tail $O/bench$3.err; exit 1; }
  cat $O/bench$3.json ;;
rehearse)
  for cfg in "2" "3" "4 --grid4 32" "5" "6"; do
    t=${cfg%% *}
    timeout -k 10 300 python bench.py --gpus 2 --backend gloo --steps 5 --warmup 1 --config $cfg > $O/n2_cfg$t.json 2> $O/n2_cfg$t.err || { echo "rehearsal cfg$t failed"; tail -20 $O/n2_cfg$t.err; exit 1; }
    echo "cfg$t: $(cut -c1-300 $O/n2_cfg$t.json)"
  done ;;
prof)
  for CFG in ${3:-2 3}; do
    case $CFG in 4) A="--steps 3 --warmup 1";; 3|6) A="--steps 20 --warmup 3";; *) A="--steps 50 --warmup 5";; esac
    PROF $O/prof_cfg$CFG "" 400 -- python3 $R/bench.py --config $CFG $A --no-cpu-baseline --no-projection > $O/bench_cfg$CFG.json 2> $O/bench_cfg$CFG.err || { echo "prof cfg$CFG failed"; tail $O/bench_cfg$CFG.err; exit 1; }
    echo "prof cfg$CFG ok"
  done ;;
pmc)
  CFG=${3:-2}; i=0
  for set in "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU" \
             "SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_SMEM" \
             "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    PROF $O/c${CFG}p$i "$set" 150 -- python3 $R/bench.py --config $CFG --no-cpu-baseline --no-projection --steps 3 --warmup 1 > $O/c${CFG}p$i.json 2> $O/c${CFG}p$i.err || { echo "pmc pass $i failed"; tail $O/c${CFG}p$i.err; exit 1; }
  done
  python3 scripts/pmc_summary.py $O/c${CFG}p1 $O/c${CFG}p2 > $O/pmc_summary_cfg$CFG.txt || exit 1
  mkdir -p $O/t && cp -r $O/c${CFG}p3 $O/t/c${CFG}p7 && cp -r $O/c${CFG}p4 $O/t/c${CFG}p8
  python3 scripts/pmc_traffic.py $O/t $CFG $O/pmc_traffic_cfg$CFG.json || exit 1
  cat $O/pmc_summary_cfg$CFG.txt ;;
traffic)
  for CFG in ${3:-2 3}; do
    KN=""; [ $CFG = 4 ] && KN="k_scn<"; [ $CFG = 5 ] && KN="k_future<"
    for p in 7:FETCH_SIZE 8:WRITE_SIZE; do
      i=${p%%:*}; C=${p#*:}
      PROF $O/c${CFG}p$i "$C" 200 -- python3 $R/bench.py --config $CFG --no-cpu-baseline --no-projection --steps 2 --warmup 1 > $O/c${CFG}p$i.json 2> $O/c${CFG}p$i.err || { echo "pmc $CFG $C failed"; tail $O/c${CFG}p$i.err; exit 1; }
    done
    python3 scripts/pmc_traffic.py $O $CFG $O/pmc_traffic_cfg$CFG.json $KN || exit 1
  done ;;
wide)
  timeout -k 10 600 python scripts/wide_timing.py > $O/wide_timing.jsonl 2> $O/wide_timing.err || { echo "wide timing failed"; tail $O/wide_timing.err; exit 1; }
  cat $O/wide_timing.jsonl ;;
pmcw)
  i=0
  for set in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVES" \
             "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM" \
             "SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY" \
             "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MFMA_MOPS_F64"; do
    i=$((i+1))
    PROF $O/p$i "$set" 300 -- python3 $R/scripts/wide_timing.py > $O/p$i.jsonl 2> $O/p$i.err || { echo "pass $i failed"; tail $O/p$i.err; exit 1; }
    echo "pass $i ok"
  done
  python3 scripts/pmc_summary.py $O/p* > $O/pmc_summary_wide.txt; cat $O/pmc_summary_wide.txt | cut -c1-200 ;;
sweep)
  V="$3"
  timeout -k 10 600 python scripts/sweep_forward.py --configs ${4:-2,3} --steps 100 --variants "$V;$V" > $O/sweep.jsonl 2> $O/sweep.err || { echo "sweep failed"; tail $O/sweep.err; exit 1; }
  cat $O/sweep.jsonl ;;
diag)
  timeout -k 10 300 python scripts/sweep_forward.py --configs ${3:-2,3} --diag --variants "MDP_JIT=1" --steps 30 > $O/diag.txt 2>&1 || { echo "diag failed"; tail $O/diag.txt; exit 1; }
  cat $O/diag.txt ;;
ubench)
  make -s -C scripts/ubench $3 || exit 1
  timeout -k 10 120 ./scripts/ubench/$3 > $O/$3.txt 2>&1 || { echo "ubench $3 failed"; tail $O/$3.txt; exit 1; }
  cat $O/$3.txt ;;
*) echo "usage: scripts/gpu.sh <mode> [tag] [args]"; exit 2 ;;
esac
