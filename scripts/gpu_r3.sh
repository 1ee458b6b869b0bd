#!/bin/bash
# Round-3 GPU check: host CPU facts, the new parity tests first, then the
# whole GPU suite and short bench lines of configs 2 and 3.
# Usage: scripts/gpu_r3.sh <outdir-name> [pytest -k expression for the first pass]
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3}
mkdir -p $O
cd $R
{
  echo "nproc=$(nproc) OMP_NUM_THREADS=$OMP_NUM_THREADS"
  cat /sys/fs/cgroup/cpu.max 2>/dev/null | sed 's/^/cpu.max=/'
  python -c "import os; print('affinity', len(os.sched_getaffinity(0)))"
  lscpu | grep -E "^(Model name|Socket|Core|Thread|CPU\(s\))"
} > $O/host.txt 2>&1
K=${2:-}
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "$K" > $O/pytest_new.log 2>&1
  rc=$?; tail -5 $O/pytest_new.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for c in 2 3 6; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 50 --warmup 5 > $O/bench_cfg$c.json 2> $O/bench_cfg$c.err || { echo "bench $c failed"; tail $O/bench_cfg$c.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/bench_cfg$c.json')); print($c, 'step_ms', d['ms_per_step'], 'kernels', d['kernel_ms'], 'frac', d['roofline']['frac'])"
done
# config 6 on the generic runtime-shape kernels, for the per-use comparison
MDP_JIT=0 timeout -k 10 300 python bench.py --config 6 --no-cpu-baseline --steps 10 --warmup 2 > $O/bench_cfg6_generic.json 2> $O/bench_cfg6_generic.err || { echo "bench 6 generic failed"; tail $O/bench_cfg6_generic.err; exit 1; }
python -c "import json,sys; d=json.load(open('$O/bench_cfg6_generic.json')); print('6-generic', 'step_ms', d['ms_per_step'], 'kernels', d['kernel_ms'])"
