"""Summarise rocprofv3 --pmc CSVs per kernel: python scripts/pmc_summary.py gpurun_out/pmc/c3p*"""
import collections
import csv
import re
import sys
from pathlib import Path


def short(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    return re.split(r"\(", n)[0]


agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    f = Path(d) / "run_counter_collection.csv"
    if not f.exists():
        continue
    for r in csv.DictReader(open(f)):
        agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, dd in agg.items():
    if "rocclr" in k:
        continue
    print(k)
    for c, v in sorted(dd.items()):
        print(f"    {c:28s} {sum(v) / len(v):16.1f}   (n={len(v)})")
