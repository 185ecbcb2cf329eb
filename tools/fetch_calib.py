"""Combine the fetch_calib runs (tools/fetch_calib.hip) into the counter factors:
per record shape and table size, the counters of the measured dispatch (rep 1)
over its exact algorithmic bytes.  usage: python tools/fetch_calib.py <gpu_batch out dir>"""
import csv
import json
import os
import sys

out = sys.argv[1]
runs = [json.loads(line) for line in open(os.path.join(out, "calib_plain.log")) if line.startswith("{")]
counters = {}
for group in ("calib_fetch", "calib_rdreq", "calib_dram"):
    for root, _, files in os.walk(os.path.join(out, group)):
        for f in files:
            if f.endswith("counter_collection.csv"):
                for row in csv.DictReader(open(os.path.join(root, f))):
                    if "gather<" not in row["Kernel_Name"]:
                        continue  # the table fills (hipMemset) are dispatches too
                    d = int(row["Dispatch_Id"])
                    counters.setdefault(d, {})
                    counters[d][row["Counter_Name"]] = counters[d].get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
ids = sorted(counters)
assert len(ids) == len(runs), (len(ids), len(runs))
table = []
for run, d in zip(runs, ids):
    c = counters[d]
    algo = run["algo_bytes"]
    row = dict(run)
    row["FETCH_SIZE_KiB"] = c.get("FETCH_SIZE")
    row["fetch_x1024_over_algo"] = c["FETCH_SIZE"] * 1024.0 / algo if "FETCH_SIZE" in c else None
    rq = {k: c.get(f"TCC_EA0_RDREQ{k}_sum") for k in ("", "_32B", "_64B", "_128B")}
    row.update({f"RDREQ{k}": v for k, v in rq.items()})
    if rq["_32B"] is not None and rq["_64B"] is not None and rq["_128B"] is not None:
        # bytes the memory side was asked for: sized requests (a request not in the sized
        # counters is taken as 64 B)
        sized = 32.0 * rq["_32B"] + 64.0 * rq["_64B"] + 128.0 * rq["_128B"]
        rest = max(0.0, rq[""] - rq["_32B"] - rq["_64B"] - rq["_128B"])
        row["req_bytes"] = sized + 64.0 * rest
        row["req_bytes_over_algo"] = row["req_bytes"] / algo
    row["RDREQ_DRAM"] = c.get("TCC_EA0_RDREQ_DRAM_sum")
    hit, miss = c.get("TCC_HIT_sum"), c.get("TCC_MISS_sum")
    row["L2_hit"] = hit / (hit + miss) if hit is not None and miss else None
    table.append(row)
    print(json.dumps(row))
measured = [r for r in table if r["rep"] == 1]
print("\nrecord  table   fetchx1024/algo  req_bytes/algo  RDREQ_DRAM/RDREQ  L2 hit  GB/s")
for r in measured:
    dr = r["RDREQ_DRAM"] / r["RDREQ"] if r.get("RDREQ_DRAM") is not None and r.get("RDREQ") else float("nan")
    print(f"{r['record_bytes']:>6}  {r['table']:>6}  {r['fetch_x1024_over_algo']:>15.3f}  "
          f"{r.get('req_bytes_over_algo', float('nan')):>14.3f}  {dr:>16.3f}  {r['L2_hit'] or 0:>6.3f}  {r['GBps']:>6.0f}")
