#!/bin/bash
# Kernel-trace + stats profile of the default bench (and config 3), then PMC passes.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof
cd /tmp && export TMPDIR=/tmp
for CFG in 2 3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof/cfg$CFG -o run -- python3 $R/bench.py --config $CFG --steps 50 --warmup 5 > $R/gpurun_out/prof/bench_cfg$CFG.json 2> $R/gpurun_out/prof/bench_cfg$CFG.err || { echo "prof cfg$CFG failed"; tail $R/gpurun_out/prof/bench_cfg$CFG.err; exit 1; }
  echo "prof cfg$CFG ok"
done
[ "${PMC:-1}" = 0 ] || bash $R/scripts/gpu_pmc.sh ${PMC_CFG:-2}
