set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc4
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU" "SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVES"; do
  i=$((i+1))
  timeout -k 10 150 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/c4p$i -o run -- python3 $R/bench.py --config 4 --grid4 96 --no-cpu-baseline --steps 2 --warmup 1 > $O/c4p$i.json 2> $O/c4p$i.err || { echo "pass $i failed"; tail -5 $O/c4p$i.err; exit 1; }
done
python3 $R/scripts/pmc_summary.py $O/c4p1 $O/c4p2
