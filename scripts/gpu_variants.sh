#!/bin/bash
# A/B bench lines of engine knob variants: $1 = configs (e.g. "2 3"),
# $2 = ';'-separated variants, each a space-separated list of VAR=value
# ("-" = defaults); every variant runs twice, interleaved.
# Output: gpurun_out/variants/
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/variants
mkdir -p $O
cd $R
IFS=';' read -ra VARS <<< "$2"
for rep in 1 2; do
  for c in $1; do
    i=0
    for v in "${VARS[@]}"; do
      i=$((i+1))
      [ "$v" = "-" ] && v=""
      env $v timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 200 --warmup 10 > $O/c${c}_v${i}_r$rep.json 2> $O/c${c}_v${i}_r$rep.err || { echo "bench $c [$v] failed"; tail $O/c${c}_v${i}_r$rep.err; exit 1; }
      python -c "import json; d=json.load(open('$O/c${c}_v${i}_r$rep.json')); print($c, '[$v]', 'step_us %.2f' % (d['ms_per_step']*1e3), 'kernels', {k: round(x*1e3, 2) for k, x in d['kernel_ms'].items()}, 'parity', d.get('parity', {}).get('max_rel_dposterior'))"
    done
  done
done
