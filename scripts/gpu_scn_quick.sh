#!/bin/bash
# scenario engine quick check: parity tests then the config-4 bench (64^3 and 256^3)
set -o pipefail
mkdir -p gpurun_out/scnq
O=gpurun_out/scnq
timeout -k 10 300 python -u -m pytest tests/test_gpu_scenario.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python bench.py --config 4 --grid4 64 --steps 3 --warmup 1 --no-cpu-baseline > $O/b64.json 2> $O/b64.err || { echo "bench64 failed"; tail $O/b64.err; exit 1; }
timeout -k 10 300 python bench.py --config 4 --steps 3 --warmup 1 > $O/b256.json 2> $O/b256.err || { echo "bench256 failed"; tail $O/b256.err; exit 1; }
python -c "
import json
for f in ['$O/b64.json','$O/b256.json']:
    d=json.load(open(f)); print(f, round(d['ms_per_step'],3), d['kernel_ms'], round(d['roofline']['frac'],4), d.get('parity'))
"
