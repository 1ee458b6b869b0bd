#!/bin/bash
# GPU test suite (optionally a subset: $1 = pytest -k expression) and short
# bench lines of configs 2 and 3.  Output: gpurun_out/quick/
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/quick
mkdir -p $O
cd $R
K=${1:-}
if [ -n "$K" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -k "$K" > $O/pytest.log 2>&1
else
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
fi
rc=$?; tail -15 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for c in 2 3; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 50 --warmup 5 > $O/bench_cfg$c.json 2> $O/bench_cfg$c.err || { echo "bench $c failed"; tail $O/bench_cfg$c.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/bench_cfg$c.json')); print($c, 'step_ms', d['ms_per_step'], 'kernels', d['kernel_ms'], 'frac', d['roofline']['frac'])"
done
