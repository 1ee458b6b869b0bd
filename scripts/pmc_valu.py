"""VALU instructions per launch of k_future from a rocprofv3 --pmc pass
(SQ_INSTS_VALU, wave-instructions) for bench.py's VALU-issue roofline.

usage: python scripts/pmc_valu.py <pass dir> <replicates> <years> <out.json>
"""
import csv
import json
import sys
from pathlib import Path

d, nrep, years, out = Path(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), Path(sys.argv[4])
rows = [r for r in csv.DictReader(open(d / "run_counter_collection.csv"))
        if r["Counter_Name"] == "SQ_INSTS_VALU" and "k_future<" in r["Kernel_Name"]]
v = [float(r["Counter_Value"]) for r in rows]
res = {"kernel": "k_future", "replicates": nrep, "years": years,
       "valu_insts_per_launch": sum(v) / len(v), "dispatches": len(v),
       "unit": "wave64 VALU instructions (SQ_INSTS_VALU, summed over the chip)"}
out.write_text(json.dumps(res, indent=1) + "\n")
print(json.dumps(res))
