#!/bin/bash
# zexp A/B: parity tests of the likelihood engine, then config-2/3 bench with and without in-LDS S expansion
set -o pipefail
mkdir -p gpurun_out/zexp
O=gpurun_out/zexp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit 1
for z in 1 0; do
  MDP_ZEXP=$z timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > $O/cfg2_z$z.json 2> $O/cfg2_z$z.err || { echo "bench z=$z failed"; tail $O/cfg2_z$z.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/cfg2_z$z.json')); print('z=$z', d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'], d.get('parity'))"
done
