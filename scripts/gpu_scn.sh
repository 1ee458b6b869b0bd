#!/bin/bash
# GPU check of the scenario engine: parity tests, config-4 bench (small, full), rocprof stats.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/scn
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_scenario.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/scn/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/scn/pytest.log; exit 1; }
tail -3 gpurun_out/scn/pytest.log
timeout -k 10 120 python bench.py --config 4 --grid4 64 --steps 3 --warmup 1 > gpurun_out/scn/bench4_64.json 2> gpurun_out/scn/bench4_64.err || { echo "bench64 failed"; tail gpurun_out/scn/bench4_64.err; exit 1; }
cat gpurun_out/scn/bench4_64.json
timeout -k 10 300 python bench.py --config 4 --steps 3 --warmup 1 > gpurun_out/scn/bench4.json 2> gpurun_out/scn/bench4.err || { echo "bench256 failed"; tail gpurun_out/scn/bench4.err; exit 1; }
cat gpurun_out/scn/bench4.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/scn/prof -o run -- python3 $R/bench.py --config 4 --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/scn/prof_bench4.json 2> $R/gpurun_out/scn/prof.err || { echo "prof failed"; tail $R/gpurun_out/scn/prof.err; exit 1; }
echo prof ok
