#!/bin/bash
# PMC passes (one counter group per run, kernel-trace only) on bench config $1.
# Stops at the first failing pass.
set -o pipefail
CFG=${1:-3}
EXTRA=${2:-}        # extra bench.py flags, e.g. "--grid4 64"
NPASS=${3:-8}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS" "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM" "GRBM_GUI_ACTIVE GRBM_COUNT" "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 150 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $R/gpurun_out/pmc/c${CFG}p$i -o run -- python3 $R/bench.py --config $CFG $EXTRA --no-cpu-baseline --steps 3 --warmup 1 > $R/gpurun_out/pmc/c${CFG}p$i.json 2> $R/gpurun_out/pmc/c${CFG}p$i.err
  rc=$?
  echo "pmc pass $i ($set) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  [ $i -ge $NPASS ] && break
done
