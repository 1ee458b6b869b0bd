#!/bin/bash
# PMC passes on bench config $2 for each ';'-separated engine variant $3
# (env assignments, comma-separated), output gpurun_out/$1/<v>p<i>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-pmcv}
CFG=${2:-2}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
v=0
IFS=';' read -ra VARS <<< "$3"
for var in "${VARS[@]}"; do
  v=$((v+1))
  i=0
  for set in "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_WAVES" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" "SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"; do
    i=$((i+1))
    env $(echo $var | tr ',' ' ') timeout -k 10 150 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/v${v}p$i -o run -- python3 $R/bench.py --config $CFG --no-cpu-baseline --steps 3 --warmup 1 > $O/v${v}p$i.json 2> $O/v${v}p$i.err
    rc=$?
    echo "variant $v ($var) pass $i rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
  echo "== variant $v: $var"
  python3 $R/scripts/pmc_summary.py $O/v${v}p* | grep -A20 mdp_fwd_jit | head -16
done
