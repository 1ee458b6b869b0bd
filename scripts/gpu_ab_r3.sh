#!/bin/bash
# A/B of the round-3 tree (_r3, a git worktree built in-tree) against HEAD on
# one box: config-2 bench lines alternating, then HEAD variants.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-abr3}
mkdir -p $O
cd $R
for i in 1 2 3; do
  (cd _r3 && timeout -k 10 120 python bench.py --config 2 --no-cpu-baseline --steps 200 --warmup 20) > $O/r3_$i.json 2>$O/r3_$i.err || { tail $O/r3_$i.err; exit 1; }
  timeout -k 10 120 python bench.py --config 2 --no-cpu-baseline --steps 200 --warmup 20 > $O/head_$i.json 2>$O/head_$i.err || { tail $O/head_$i.err; exit 1; }
  python -c "import json; a=json.load(open('$O/r3_$i.json')); b=json.load(open('$O/head_$i.json')); print('r3', a['ms_per_step']*1e3, a['kernel_ms'], 'head', b['ms_per_step']*1e3, b['kernel_ms'])"
done
timeout -k 10 300 python scripts/sweep_forward.py --configs 2 --steps 100 --variants "MDP_JIT=1;MDP_FUSED_SBUILD=0;MDP_JIT=1;MDP_FUSED_SBUILD=0" > $O/sweep.jsonl 2> $O/sweep.err || { tail $O/sweep.err; exit 1; }
cut -c1-200 $O/sweep.jsonl
