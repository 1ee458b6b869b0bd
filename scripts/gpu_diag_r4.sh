#!/bin/bash
# Phase stamps (diag library) of config-2/3 variants: $1 = output dir,
# $2 = configs, $3 = ';'-separated variants
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-diag4}
mkdir -p $O
cd $R
timeout -k 10 400 python scripts/sweep_forward.py --configs ${2:-2} --steps 50 --variants "$3" --diag > $O/diag.txt 2>&1 || { echo "diag failed"; tail $O/diag.txt; exit 1; }
grep -v amdgpu.ids $O/diag.txt | grep -v "after idle" | cut -c1-1500
