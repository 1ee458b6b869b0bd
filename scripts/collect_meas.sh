#!/bin/bash
# Copy the judged summaries of a gpu_measure.sh run into profiles/<name>/ and
# refresh the PMC files bench.py reads (profiles/pmc_*.json).
set -e
M=gpurun_out/meas
D=profiles/$1
mkdir -p $D
cp $M/bench_cfg2.json $D/bench_default.json
for c in 2 3 4 5 6; do
  cp $M/prof_bench_cfg$c.json $D/bench_cfg$c.json
  cp $M/prof_cfg$c/run_kernel_stats.csv $D/rocprof_kernel_stats_cfg$c.csv
done
cp $M/pmc_summary_cfg2.txt $M/pmc_summary_cfg3.txt $M/pmc_traffic_cfg*.json $M/pmc_valu_cfg5.json $D/
cp $M/pmc_traffic_cfg*.json $M/pmc_valu_cfg5.json profiles/
cp $M/sweep_cfg6.jsonl $M/wide_timing.jsonl $D/
