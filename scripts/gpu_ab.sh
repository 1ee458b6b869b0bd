#!/bin/bash
# A/B sweep of engine variants (alternating, twice) on one box, then the
# phase stamps of each.  $1 = output dir name, $2 = configs, $3 = variants
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-ab}
mkdir -p $O
cd $R
V="$3"
timeout -k 10 400 python scripts/sweep_forward.py --configs ${2:-2} --steps 100 --variants "$V;$V" > $O/sweep.jsonl 2> $O/sweep.err || { echo "sweep failed"; tail $O/sweep.err; exit 1; }
cut -c1-220 $O/sweep.jsonl
timeout -k 10 300 python scripts/sweep_forward.py --configs ${2:-2} --steps 30 --variants "$V" --diag > $O/diag.txt 2>&1 || { echo "diag failed"; tail $O/diag.txt; exit 1; }
grep -E "variant|back to back|k_forward\(jit\)|k_qrows:" $O/diag.txt | grep -v "after idle" | cut -c1-330
