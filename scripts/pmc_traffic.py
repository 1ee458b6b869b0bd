"""HBM traffic per launch of a kernel from rocprofv3 PMC passes.

usage: python scripts/pmc_traffic.py <pmc dir> <config> <out.json> [kernel]
(kernel: a substring of the kernel name, default mdp_fwd_jit)
Reads <dir>/c<config>p7 (FETCH_SIZE) and p8 (WRITE_SIZE) kernel CSVs (see
scripts/gpu_pmc.sh).  Corrections per MI355X_MICROARCH.md (HBM section):
FETCH_SIZE reports half the bytes of wide coalesced reads on gfx950 -> x2;
WRITE_SIZE is exact for 16-byte streaming stores.  Both are in KiB.
"""
import csv
import json
import sys
from pathlib import Path

d, cfg, out = Path(sys.argv[1]), sys.argv[2], Path(sys.argv[3])
KERNEL = sys.argv[4] if len(sys.argv) > 4 else "mdp_fwd_jit"


def mean(pas, counter, kernel=KERNEL):
    """Mean over the kernel's dispatches with the largest grid (the scenario
    kernel runs as a small v pass and the large likelihood pass)."""
    f = d / f"c{cfg}p{pas}" / "run_counter_collection.csv"
    rows = [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == counter and kernel in r["Kernel_Name"]]
    if rows and "Grid_Size" in rows[0]:
        g = max(int(r["Grid_Size"]) for r in rows)
        rows = [r for r in rows if int(r["Grid_Size"]) == g]
    v = [float(r["Counter_Value"]) for r in rows]
    return sum(v) / len(v), len(v)


fetch, n1 = mean(7, "FETCH_SIZE")
write, n2 = mean(8, "WRITE_SIZE")
res = {
    "kernel": KERNEL,
    "config": int(cfg),
    "fetch_size_kib": fetch,
    "write_size_kib": write,
    "hbm_bytes_per_launch": (2.0 * fetch + write) * 1024.0,
    "dispatches": [n1, n2],
    "correction": "FETCH_SIZE x2 (gfx950 reports half of wide coalesced reads), WRITE_SIZE as is",
}
out.write_text(json.dumps(res, indent=1) + "\n")
print(json.dumps(res))
