#!/bin/bash
# Output-layout check (CE = EC transposed on every path) and the config-2/3
# bench lines in both layouts (alternating, the first pair a warm-up).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3lay}; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_layout.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for L in ce ec; do
    timeout -k 10 120 python bench.py --config 2 --layout $L --no-cpu-baseline --steps 200 --warmup 20 >> $O/bench2.jsonl 2>> $O/bench.err || exit 1
  done
done
for L in ce ec; do
  timeout -k 10 200 python bench.py --config 3 --layout $L --no-cpu-baseline --steps 50 --warmup 5 >> $O/bench3.jsonl 2>> $O/bench.err || exit 1
done
