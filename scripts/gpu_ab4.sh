#!/bin/bash
# A/B of engine variants on one box: parity subset ($2, "-" to skip), then a
# sweep alternating the ';'-separated variants $3 twice over configs $4,
# then the phase stamps of each on config 2.  Output gpurun_out/$1/
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-ab4}
mkdir -p $O
cd $R
T=${2:--}
if [ "$T" != "-" ]; then
  timeout -k 10 600 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
  rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
V="$3"
timeout -k 10 500 python scripts/sweep_forward.py --configs ${4:-2,3} --steps 100 --variants "$V;$V" > $O/sweep.jsonl 2> $O/sweep.err || { echo "sweep failed"; tail $O/sweep.err; exit 1; }
python - $O/sweep.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["config"], d["variant"], {k: d[k] for k in d if k.startswith("k_")}, "step", d["step_us"], "same_inf", d["same_inf"], "dlog", d["max_dlog_vs_first"])
PY
if [ -n "$5" ]; then
  timeout -k 10 300 python scripts/sweep_forward.py --configs 2 --steps 30 --variants "$V" --diag > $O/diag.txt 2>&1 || { echo "diag failed"; tail $O/diag.txt; exit 1; }
  grep -E "variant|back to back|k_forward\(jit\)" $O/diag.txt | grep -v "after idle" | cut -c1-330
fi
