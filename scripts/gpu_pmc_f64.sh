#!/bin/bash
# FP64 instruction counts (one PMC pass, kernel-trace only) of bench configs
# 2, 3 and 6: executed flops = 64 x (2 FMA + MUL + ADD) wave-instructions per
# launch, against the line's flop_min.  Output gpurun_out/r5/pmcf64/.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5/pmcf64
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for CFG in ${CFGS:-2 3 6}; do
  timeout -k 10 150 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 --kernel-trace --output-format csv -d $O/c$CFG -o run -- python3 $R/bench.py --config $CFG --no-cpu-baseline --steps 3 --warmup 1 > $O/c$CFG.json 2> $O/c$CFG.err
  rc=$?
  echo "pmc f64 cfg$CFG rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
