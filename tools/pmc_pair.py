"""Side-by-side PMC summary of the timed path/sort kernel launch in rocprofv3 counter
CSVs (the last dispatch of the kernel in each directory), per segment.

    python tools/pmc_pair.py SEGMENTS dirA [dirB ...]
"""
import csv
import os
import sys


def counters(d):
    rows = []
    for root, _, files in os.walk(d):
        for f in files:
            if f.endswith("counter_collection.csv"):
                rows += [r for r in csv.DictReader(open(os.path.join(root, f)))
                         if "path_kernel<false" in r["Kernel_Name"]]
    last = max(int(r["Dispatch_Id"]) for r in rows)
    out = {}
    for r in rows:
        if int(r["Dispatch_Id"]) == last:
            out[r["Counter_Name"]] = out.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            out["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return out


segs = float(sys.argv[1])
for d in sys.argv[2:]:
    c = counters(d)
    line = {k: round(v / segs, 2) for k, v in sorted(c.items()) if not k.startswith("_")}
    if "SQ_THREAD_CYCLES_VALU" in c:
        line["lanes"] = round(c["SQ_THREAD_CYCLES_VALU"] / c["SQ_ACTIVE_INST_VALU"], 1)
    print(d, "ms", round(c["_ns"] / 1e6, 2), line)
