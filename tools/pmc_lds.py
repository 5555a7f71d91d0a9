"""Per-kernel LDS counters of one rocprofv3 --pmc pass (SQ_LDS_BANK_CONFLICT, SQ_LDS_IDX_ACTIVE,
SQ_INSTS_LDS, SQ_WAIT_INST_LDS): per-dispatch averages and the conflict share of the LDS-array
cycles.  python3 tools/pmc_lds.py <rocprofv3 output dir>"""
import csv
import glob
import json
import sys
from collections import defaultdict

per = defaultdict(lambda: defaultdict(float))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        per[(name, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
agg = defaultdict(lambda: defaultdict(list))
for (name, _), cs in per.items():
    for c, v in cs.items():
        agg[name][c].append(v)
out = {}
for name, cs in agg.items():
    e = {c: sum(v) / len(v) for c, v in cs.items()}
    if e.get("SQ_LDS_IDX_ACTIVE"):
        e["conflict_share"] = e.get("SQ_LDS_BANK_CONFLICT", 0.0) / e["SQ_LDS_IDX_ACTIVE"]
    e["dispatches"] = len(next(iter(cs.values())))
    out[name] = e
print(json.dumps(out, indent=1))
