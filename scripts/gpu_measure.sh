#!/bin/bash
# Measurement set: bench lines of configs 2-6, rocprofv3 kernel stats,
# PMC passes (FP64 instruction mix, stalls, LDS conflicts, HBM traffic) of
# configs 2 and 3, VALU count of config 5, the long-series and wide-year
# timings.  Output: gpurun_out/meas/
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/meas
mkdir -p $O/pmc
cd $R
timeout -k 10 300 python bench.py > $O/bench_cfg2.json 2> $O/bench_cfg2.err || { echo "bench cfg2 failed"; tail $O/bench_cfg2.err; exit 1; }
echo "bench cfg2 ok"
cd /tmp && export TMPDIR=/tmp
for spec in "2:--steps 50 --warmup 5" "3:--steps 20 --warmup 3" "4:--steps 3 --warmup 1" "5:--steps 20 --warmup 3" "6:--steps 10 --warmup 2"; do
  CFG=${spec%%:*}; ARGS=${spec#*:}
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cfg$CFG -o run -- python3 $R/bench.py --config $CFG $ARGS --no-cpu-baseline > $O/prof_bench_cfg$CFG.json 2> $O/prof_bench_cfg$CFG.err || { echo "prof cfg$CFG failed"; tail $O/prof_bench_cfg$CFG.err; exit 1; }
  echo "prof cfg$CFG ok"
done
for CFG in 2 3; do
  i=0
  for set in "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS" "SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVES" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -k 10 150 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/pmc/c${CFG}p$i -o run -- python3 $R/bench.py --config $CFG --no-cpu-baseline --steps 3 --warmup 1 > $O/pmc/c${CFG}p$i.json 2> $O/pmc/c${CFG}p$i.err || { echo "pmc $CFG $i failed"; tail $O/pmc/c${CFG}p$i.err; exit 1; }
  done
  mkdir -p $O/pmc/t$CFG && ln -sf $O/pmc/c${CFG}p3 $O/pmc/t$CFG/c${CFG}p7 && ln -sf $O/pmc/c${CFG}p4 $O/pmc/t$CFG/c${CFG}p8
  python3 $R/scripts/pmc_traffic.py $O/pmc/t$CFG $CFG $O/pmc_traffic_cfg$CFG.json || exit 1
  python3 $R/scripts/pmc_summary.py $O/pmc/c${CFG}p1 $O/pmc/c${CFG}p2 > $O/pmc_summary_cfg$CFG.txt || exit 1
  echo "pmc cfg$CFG ok"
done
for spec in "4:k_scn<" "5:k_future<"; do
  CFG=${spec%%:*}; KN=${spec#*:}
  for p in 7:FETCH_SIZE 8:WRITE_SIZE; do
    i=${p%%:*}; C=${p#*:}
    timeout -k 10 200 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/pmc/c${CFG}p$i -o run -- python3 $R/bench.py --config $CFG --no-cpu-baseline --steps 2 --warmup 1 > $O/pmc/c${CFG}p$i.json 2> $O/pmc/c${CFG}p$i.err || { echo "pmc $CFG $C failed"; tail $O/pmc/c${CFG}p$i.err; exit 1; }
  done
  python3 $R/scripts/pmc_traffic.py $O/pmc $CFG $O/pmc_traffic_cfg$CFG.json "$KN" || exit 1
  echo "pmc traffic cfg$CFG ok"
done
timeout -k 10 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_CVT --kernel-trace --output-format csv -d $O/pmc/c5p1 -o run -- python3 $R/bench.py --config 5 --no-cpu-baseline --steps 3 --warmup 1 > $O/pmc/c5p1.json 2> $O/pmc/c5p1.err || { echo "pmc 5 failed"; exit 1; }
python3 $R/scripts/pmc_valu.py $O/pmc/c5p1 1000000 50 $O/pmc_valu_cfg5.json || exit 1
# long series (chunked) against the generic kernels, and the wide-year paths
(cd $R && timeout -k 10 300 python scripts/sweep_forward.py --configs 6 --steps 20 --variants "MDP_JIT=1;MDP_JIT=1;MDP_JIT=0" > $O/sweep_cfg6.jsonl 2> $O/sweep_cfg6.err) || { echo "sweep cfg6 failed"; exit 1; }
(cd $R && WIDE_PATHS=default,wide WIDE60_PATHS=default,wideplain timeout -k 10 300 python scripts/wide_timing.py > $O/wide_timing.jsonl 2> $O/wide_timing.err) || { echo "wide timing failed"; exit 1; }
echo "all ok"
