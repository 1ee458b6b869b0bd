set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/meas45
mkdir -p $O/pmc
cd /tmp && export TMPDIR=/tmp
for spec in "4:k_scn<" "5:k_future<"; do
  CFG=${spec%%:*}; KN=${spec#*:}
  for p in 7:FETCH_SIZE 8:WRITE_SIZE; do
    i=${p%%:*}; C=${p#*:}
    timeout -k 10 200 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/pmc/c${CFG}p$i -o run -- python3 $R/bench.py --config $CFG --no-cpu-baseline --steps 2 --warmup 1 > $O/pmc/c${CFG}p$i.json 2> $O/pmc/c${CFG}p$i.err || { echo "pmc $CFG $C failed"; tail $O/pmc/c${CFG}p$i.err; exit 1; }
  done
  python3 $R/scripts/pmc_traffic.py $O/pmc $CFG $O/pmc_traffic_cfg$CFG.json "$KN" || exit 1
done
cd $R && timeout -k 10 200 python bench.py --config 4 --no-cpu-baseline --steps 2 --warmup 1 > $O/b4.json && timeout -k 10 200 python bench.py --config 5 --no-cpu-baseline --steps 5 --warmup 1 > $O/b5.json
