"""Summarise rocprofv3 --pmc passes of the path kernel (the bench's timed dispatch:
the last path_kernel<false, ...> launch of each pass) into the DESIGN.md §4 table.
usage: python tools/pmc_summary.py DIR [DIR ...]   (each DIR holds run_counter_collection.csv)"""
import csv
import os
import sys


def last_dispatch(path):
    rows = [r for r in csv.DictReader(open(path)) if r["Kernel_Name"].startswith("void rt::path_kernel<false")]
    if not rows:
        return {}, None
    last = max(int(r["Dispatch_Id"]) for r in rows)
    sel = [r for r in rows if int(r["Dispatch_Id"]) == last]
    vals = {}
    for r in sel:
        vals[r["Counter_Name"]] = vals.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ns = int(sel[0]["End_Timestamp"]) - int(sel[0]["Start_Timestamp"])
    return vals, (ns, sel[0]["VGPR_Count"], sel[0]["SGPR_Count"], sel[0]["Scratch_Size"], sel[0]["LDS_Block_Size"])


def main():
    vals, meta = {}, None
    for d in sys.argv[1:]:
        v, m = last_dispatch(os.path.join(d, "run_counter_collection.csv"))
        vals.update(v)
        meta = meta or m
    for k in sorted(vals):
        print(f"{k:32s} {vals[k]:.4g}")
    g = vals.get
    if g("SQ_ACTIVE_INST_VALU") and g("SQ_THREAD_CYCLES_VALU"):
        print(f"active lanes per VALU instruction   {g('SQ_THREAD_CYCLES_VALU') / g('SQ_ACTIVE_INST_VALU'):.1f} / 64")
    if g("SQ_INSTS_VALU"):
        f64 = sum(g(k, 0.0) for k in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64",
                                      "SQ_INSTS_VALU_TRANS_F64"))
        if f64:
            print(f"f64 share of VALU instructions      {f64 / g('SQ_INSTS_VALU'):.2f}")
        if g("SQ_INSTS_VALU_INT32"):
            print(f"int32 share of VALU instructions    {g('SQ_INSTS_VALU_INT32') / g('SQ_INSTS_VALU'):.2f}")
    if g("TCC_HIT_sum") is not None and g("TCC_MISS_sum"):
        print(f"L2 hit rate                         {g('TCC_HIT_sum') / (g('TCC_HIT_sum') + g('TCC_MISS_sum')):.3f}")
    if g("TCP_TCC_READ_REQ_sum"):
        print(f"mean L1->L2 read latency (cycles)   {g('TCP_TCC_READ_REQ_LATENCY_sum') / g('TCP_TCC_READ_REQ_sum'):.0f}")
    if meta:
        print(f"dispatch ns / VGPR / SGPR / scratch / LDS: {meta}")


if __name__ == "__main__":
    main()
