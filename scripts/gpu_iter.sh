#!/bin/bash
# one iteration: engine parity tests, then the phase-stamp sweep and the config-2 bench line
set -o pipefail
mkdir -p gpurun_out/iter
O=gpurun_out/iter
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python scripts/sweep_forward.py --configs 2,3 --variants "${VARIANTS:-MDP_JIT=1}" --diag > $O/diag.txt 2>&1 || { echo "diag failed"; tail $O/diag.txt; exit 1; }
grep -v amdgpu.ids $O/diag.txt
timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > $O/cfg2.json 2> $O/cfg2.err || { echo "bench failed"; tail $O/cfg2.err; exit 1; }
python -c "import json; d=json.load(open('$O/cfg2.json')); print('cfg2', d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'])"
timeout -k 10 200 python bench.py --config 3 --steps 20 --warmup 3 --no-cpu-baseline > $O/cfg3.json 2> $O/cfg3.err || { echo "bench3 failed"; tail $O/cfg3.err; exit 1; }
python -c "import json; d=json.load(open('$O/cfg3.json')); print('cfg3', d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'])"
