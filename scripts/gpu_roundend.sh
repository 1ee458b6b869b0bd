#!/bin/bash
# Round-end evidence, part $1:
#   tests : the whole GPU test suite + smoke()
#   prof  : rocprofv3 --kernel-trace --stats of every bench config, the
#           FETCH/WRITE PMC passes of configs 2 and 3, the default bench line
#   pmc   : only the PMC passes and the default bench line
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/roundend
mkdir -p $O
cd $R
if [ "$1" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
  rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
  cat $O/smoke.log
  exit 0
fi
mkdir -p $O/pmc
cd /tmp && export TMPDIR=/tmp
[ "$1" = pmc ] || for spec in "2:--steps 50 --warmup 5" "3:--steps 20 --warmup 3" "4:--steps 3 --warmup 1" "5:--steps 20 --warmup 3"; do
  CFG=${spec%%:*}; ARGS=${spec#*:}
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cfg$CFG -o run -- python3 $R/bench.py --config $CFG $ARGS > $O/bench_cfg$CFG.json 2> $O/bench_cfg$CFG.err || { echo "prof cfg$CFG failed"; tail $O/bench_cfg$CFG.err; exit 1; }
  echo "prof cfg$CFG ok"
done
for CFG in 2 3; do
  for p in 7:FETCH_SIZE 8:WRITE_SIZE; do
    i=${p%%:*}; C=${p#*:}
    timeout -k 10 150 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/pmc/c${CFG}p$i -o run -- python3 $R/bench.py --config $CFG --no-cpu-baseline --steps 3 --warmup 1 > $O/pmc/c${CFG}p$i.json 2> $O/pmc/c${CFG}p$i.err || { echo "pmc $CFG $C failed"; exit 1; }
  done
  python3 $R/scripts/pmc_traffic.py $O/pmc $CFG $O/pmc_traffic_cfg$CFG.json || exit 1
done
cd $R
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench failed"; tail $O/bench_default.err; exit 1; }
cat $O/bench_default.json
