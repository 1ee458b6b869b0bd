#!/bin/bash
# PMC passes over scripts/wide_timing.py (cases $2, paths $3 as WIDE_PATHS /
# WIDE60_PATHS want them): the wide kernels' MFMA busy, wait and LDS counters.
# Output gpurun_out/$1/p<i>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-pmcw}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVES" "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM" "SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  WIDE_PATHS=$2 WIDE60_PATHS=$3 timeout -k 10 200 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/p$i -o run -- python3 $R/scripts/wide_timing.py > $O/p$i.jsonl 2> $O/p$i.err
  rc=$?
  echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 $R/scripts/pmc_summary.py $O/p* | grep -A20 k_fwd_mma | head -24
