#!/bin/bash
# GPU perf round: variant sweep, counter list, PMC passes on k_forward (config 3)
set -o pipefail
mkdir -p gpurun_out/pmc
timeout -k 10 200 python scripts/sweep_forward.py > gpurun_out/sweep.jsonl 2> gpurun_out/sweep.err || { echo "sweep failed"; tail gpurun_out/sweep.err; exit 1; }
cat gpurun_out/sweep.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/pmc/counters.txt 2>&1
R=$GRAFT_REPO_ROOT
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $R/gpurun_out/pmc/p$i -o run -- python3 $R/bench.py --config 3 --no-cpu-baseline --steps 3 --warmup 1 > $R/gpurun_out/pmc/p$i.json 2> $R/gpurun_out/pmc/p$i.err
  echo "pmc pass $i ($set) rc=$?"
done
