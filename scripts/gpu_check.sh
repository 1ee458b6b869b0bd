#!/bin/bash
# GPU round script: parity tests, variant sweep (+diag stamps), bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python scripts/sweep_forward.py > gpurun_out/sweep.jsonl 2> gpurun_out/sweep.err || { echo "sweep failed"; tail gpurun_out/sweep.err; exit 1; }
cat gpurun_out/sweep.jsonl
timeout -k 10 200 python scripts/sweep_forward.py --variants "MDP_JIT=0,MDP_EPL=2" --diag > gpurun_out/diag.txt 2>&1 || { echo "diag failed"; exit 1; }
grep -v "^{" gpurun_out/diag.txt
timeout -k 10 240 python bench.py --steps 50 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
