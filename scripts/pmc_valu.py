"""VALU work per launch of k_future from one rocprofv3 --pmc pass, for
bench.py's issue-cost roofline.

Counters (one pass, 8 SQ counters): SQ_INSTS_VALU and its classes INT64,
INT32, FMA/MUL/ADD_F64, TRANS_F64, CVT (wave-instructions summed over the
chip).  Issue cost per wave64 instruction on one SIMD, measured by
scripts/ubench/int_rates.hip: v_mad_u64_u32 (the Philox products, class
INT64) 8 cycles, v_lshl_add_u64 4, FP64 add/mul/fma 4, 32-bit ops 2.  INT64 is
priced at 8 (the Philox multiplies are most of it: 19 per Philox call against
one or two 64-bit address ops per year), CVT (to / from f64) at 4,
TRANS_F64 at 16; every other VALU instruction at 2.

usage: python scripts/pmc_valu.py <pass dir> <replicates> <years> <out.json>
"""
import collections
import csv
import json
import sys
from pathlib import Path

COST = {"SQ_INSTS_VALU_INT64": 8, "SQ_INSTS_VALU_FMA_F64": 4, "SQ_INSTS_VALU_MUL_F64": 4,
        "SQ_INSTS_VALU_ADD_F64": 4, "SQ_INSTS_VALU_CVT": 4, "SQ_INSTS_VALU_TRANS_F64": 16}
OTHER_COST = 2

d, nrep, years, out = Path(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), Path(sys.argv[4])
per = collections.defaultdict(dict)  # dispatch -> counter -> value
for r in csv.DictReader(open(d / "run_counter_collection.csv")):
    if "k_future<" in r["Kernel_Name"]:
        per[r["Dispatch_Id"]][r["Counter_Name"]] = per[r["Dispatch_Id"]].get(r["Counter_Name"], 0.0) + float(
            r["Counter_Value"])
names = sorted({c for v in per.values() for c in v})
mean = {c: sum(v.get(c, 0.0) for v in per.values()) / len(per) for c in names}
total = mean["SQ_INSTS_VALU"]
priced = sum(mean.get(c, 0.0) for c in COST)
cycles = sum(mean.get(c, 0.0) * w for c, w in COST.items()) + (total - priced) * OTHER_COST
res = {"kernel": "k_future", "replicates": nrep, "years": years, "dispatches": len(per),
       "valu_insts_per_launch": total, "classes": {c: mean[c] for c in names if c != "SQ_INSTS_VALU"},
       "issue_cycles_per_launch": cycles,
       "issue_cost": {**{c: w for c, w in COST.items()}, "other": OTHER_COST},
       "unit": "wave64 instructions / SIMD issue cycles, summed over the chip"}
out.write_text(json.dumps(res, indent=1) + "\n")
print(json.dumps(res))
