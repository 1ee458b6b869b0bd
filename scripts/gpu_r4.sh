#!/bin/bash
# Round 4 iteration: forward-path GPU tests (or $2 = pytest args), bench
# lines of configs 2 and 3, a variant sweep, and a 2-rank gloo rehearsal of
# the strong-scaling block.  Output: gpurun_out/$1/
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4}
mkdir -p $O
cd $R
T=${2:-tests/test_gpu_parity.py tests/test_gpu_layout.py tests/test_gpu_longseries.py tests/test_gpu_highvar.py}
timeout -k 10 900 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for c in 2 3; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 50 --warmup 5 > $O/bench_cfg$c.json 2> $O/bench_cfg$c.err || { echo "bench $c failed"; tail $O/bench_cfg$c.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/bench_cfg$c.json')); print($c, 'step_ms', d['ms_per_step'], 'kernels', d['kernel_ms'], 'frac', d['roofline']['frac'])"
done
timeout -k 10 300 python scripts/sweep_forward.py --configs 2,3 --steps 50 --variants "${VARIANTS:-MDP_JIT=1;MDP_EPL=2;MDP_FUSED=0}" > $O/sweep.jsonl 2> $O/sweep.err || { echo "sweep failed"; tail $O/sweep.err; exit 1; }
cut -c1-300 $O/sweep.jsonl
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 3 --config 3 --backend gloo > $O/bench_gloo2_cfg3.json 2> $O/bench_gloo2.err || { echo "gloo rehearsal failed"; tail $O/bench_gloo2.err; exit 1; }
python -c "import json; d=json.loads([l for l in open('$O/bench_gloo2_cfg3.json') if l.startswith('{')][-1]); print('gloo2', d['value'], d['job'], d['strong'])"
if [ -n "$DIAG" ]; then
  timeout -k 10 300 python scripts/sweep_forward.py --configs 2,3 --steps 30 --variants "MDP_JIT=1" --diag > $O/diag.txt 2>&1 || { echo "diag failed"; tail $O/diag.txt; exit 1; }
  grep -v amdgpu.ids $O/diag.txt | cut -c1-1500
fi
