#!/bin/bash
# Round-4 iteration: forward-path parity ($2 = pytest targets, "-" to skip),
# bench lines of configs 2 and 3, then phase stamps of $3 variants (config 2).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-it4}
mkdir -p $O
cd $R
T=${2:-tests/test_gpu_parity.py tests/test_gpu_layout.py tests/test_gpu_longseries.py tests/test_gpu_highvar.py}
if [ "$T" != "-" ]; then
  timeout -k 10 600 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
  rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
for c in 2 3; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 100 --warmup 10 > $O/bench_cfg$c.json 2> $O/bench_cfg$c.err || { echo "bench $c failed"; tail $O/bench_cfg$c.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/bench_cfg$c.json')); print($c, 'step_us', round(d['ms_per_step']*1e3,2), 'kernels_us', {k: round(v*1e3,2) for k,v in d['kernel_ms'].items()}, 'frac', round(d['roofline']['frac'],3))"
done
if [ -n "$3" ]; then
  timeout -k 10 400 python scripts/sweep_forward.py --configs ${4:-2} --steps 50 --variants "$3" --diag > $O/diag.txt 2>&1 || { echo "diag failed"; tail $O/diag.txt; exit 1; }
  grep -v amdgpu.ids $O/diag.txt | grep -v "after idle" | cut -c1-900
fi
