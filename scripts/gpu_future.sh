#!/bin/bash
# GPU check of the future engine: parity tests, config-5 bench, rocprof stats.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/fut
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_future.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/fut/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/fut/pytest.log; exit 1; }
tail -3 gpurun_out/fut/pytest.log
timeout -k 10 200 python bench.py --config 5 --steps 10 --warmup 2 > gpurun_out/fut/bench5.json 2> gpurun_out/fut/bench5.err || { echo "bench failed"; tail gpurun_out/fut/bench5.err; exit 1; }
cat gpurun_out/fut/bench5.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/fut/prof -o run -- python3 $R/bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/fut/prof_bench5.json 2> $R/gpurun_out/fut/prof.err || { echo "prof failed"; tail $R/gpurun_out/fut/prof.err; exit 1; }
echo prof ok
