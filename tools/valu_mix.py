"""Static VALU mix of the timed path-kernel instances, priced with the measured
issue costs of tools/valu_rates.hip (profiles/r04/valu_rates_full.log), so that
bench.py's VALU roofline can price the instructions its PMC classes do not name.

The PMC counters split a launch's VALU instructions into f64 FMA/MUL/ADD, f64
transcendental, int64, int32, conversions and f32 FMA/MUL/ADD/transcendental;
what is left ("rest": moves, compares, cndmask, readlane, DPP, bit ops the
hardware does not count as int32) has no counter.  Its price is the mean of the
measured costs of those opcodes, weighted by how often each appears in the
kernel's code (a static weight: the listing, not the dynamic trace — stated as
such in the bench line).

    python tools/valu_mix.py [librt_amd.so] > tools/valu_prices.json
"""
import json
import os
import re
import subprocess
import sys
import tempfile
from collections import Counter

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from kernel_regs import LLVM, code_objects  # noqa: E402

RATES = os.path.join(os.path.dirname(HERE), "profiles", "r04", "valu_rates_full.log")
# the PMC classes bench.py counts directly (opcode prefixes that belong to them)
F64 = ("v_fma_f64", "v_fmac_f64", "v_mul_f64", "v_add_f64")
TRANS64 = ("v_rcp_f64", "v_rsq_f64", "v_sqrt_f64", "v_frexp", "v_fract_f64", "v_rndne_f64", "v_trunc_f64",
           "v_floor_f64", "v_ceil_f64", "v_ldexp_f64")
# product instances (render.hip path_fn_r): C2 shape-only fused (5 waves), the compact triangle-only
# resumable kernel (C3/C4/C5), the f64 triangle-only resumable kernel
INSTANCES = {"C2": "path_kernel<false, false, 5, false, 1, false>",
             "C3": "path_kernel<false, false, 4, true, 2, true>",
             "tri_f64": "path_kernel<false, false, 4, true, 2, false>"}


def measured():
    """opcode -> cycles per wave64 instruction at 8 waves/SIMD (wall-clock form)."""
    out = {}
    for line in open(RATES):
        m = re.match(r"(v_\S+)\s+waves/SIMD 8\s+cycles/wave-instr/SIMD\s+([\d.]+)", line)
        if m:  # plain rows only ("v_cndmask_b32 (vcc)" re-wrote VCC in its loop: a test artefact)
            out.setdefault(m.group(1), float(m.group(2)))
    return out


INT32 = ("v_add_u32", "v_sub_u32", "v_subrev_u32", "v_and_b32", "v_or_b32", "v_xor_b32", "v_lshl", "v_lshr",
         "v_ashr", "v_bfe", "v_mul_lo", "v_mul_hi", "v_mad_u32", "v_add_co", "v_addc", "v_sub_co", "v_subb",
         "v_not", "v_bfi", "v_alignbit", "v_xad", "v_add3", "v_or3", "v_and_or", "v_lshl_or", "v_add_lshl",
         "v_mul_u32", "v_bcnt", "v_mbcnt", "v_bitop3")
F32 = ("v_add_f32", "v_sub_f32", "v_subrev_f32", "v_mul_f32", "v_fma_f32", "v_fmac_f32", "v_rcp_f32",
       "v_rcp_iflag_f32", "v_trunc_f32", "v_rsq_f32", "v_sqrt_f32")


def class_of(op):
    """the PMC class an opcode is counted in (bench.py valu_roofline)."""
    b = re.sub(r"_e(32|64)$", "", op)
    if b.startswith(F64):
        return "f64"
    if b.startswith(TRANS64):
        return "trans_f64"
    if b.startswith("v_cvt"):
        return "cvt"
    if b.startswith(F32):
        return "f32"
    if ("_u64" in b or "_i64" in b or b.startswith("v_lshl_add_u64")) and not b.startswith("v_cmp"):
        return "int64"
    if b.startswith(INT32):
        return "int32"
    return "rest"


def price(op, rates):
    """measured cost of an opcode: its own row, else the row of its family."""
    base = re.sub(r"_e(32|64)$", "", op)
    if base in rates:
        return rates[base], base
    fam = [("v_cmp_class", "v_cmp_class_f64"), ("v_cmp", "v_cmp_lt_f64" if "f64" in base else "v_cmp_gt_u32"),
           ("v_cndmask", "v_cndmask_b32"), ("v_mov_b64", "v_fma_f64"), ("v_mov_b32_dpp", "v_mov_b32_dpp"),
           ("v_mov", "v_mov_b32"), ("v_readfirstlane", "v_readfirstlane_b32"), ("v_readlane", "v_readfirstlane_b32"),
           ("v_writelane", "v_readfirstlane_b32"), ("v_max_f64", "v_max_f64"), ("v_min_f64", "v_max_f64"),
           ("v_max", "v_add_f32"), ("v_min", "v_add_f32"), ("v_cvt_f64", "v_cvt_f64_f32"),
           ("v_cvt", "v_cvt_f32_f64"), ("v_div_", "v_div_fmas_f64"),
           # int32 family: simple ALU ops at the v_add_u32 / v_and_b32 rate, shifts / fields /
           # multiplies / carries at the v_lshlrev_b32 / v_bfe_u32 / v_mul_lo_u32 / v_add_co_u32 rate
           ("v_sub_u32", "v_add_u32"), ("v_subrev_u32", "v_add_u32"), ("v_or_b32", "v_and_b32"),
           ("v_xor_b32", "v_and_b32"), ("v_not", "v_and_b32"), ("v_lshr", "v_lshlrev_b32"),
           ("v_ashr", "v_lshlrev_b32"), ("v_lshl", "v_lshlrev_b32"), ("v_mul", "v_mul_lo_u32"),
           ("v_mad_u32", "v_mul_lo_u32"), ("v_addc", "v_add_co_u32"), ("v_sub_co", "v_add_co_u32"),
           ("v_subb", "v_add_co_u32"), ("v_bfi", "v_bfe_u32"), ("v_alignbit", "v_bfe_u32"), ("v_bitop3", "v_bfe_u32"),
           ("v_add3", "v_bfe_u32"), ("v_bitop3_b32", "v_bitop3_b32"), ("v_xor_b32", "v_xor_b32"), ("v_or3", "v_bfe_u32"), ("v_xad", "v_bfe_u32"), ("v_and_or", "v_bfe_u32"),
           ("v_add_lshl", "v_bfe_u32"), ("v_bcnt", "v_bfe_u32"), ("v_mbcnt", "v_bfe_u32"),
           ("v_sub_f32", "v_add_f32"), ("v_subrev_f32", "v_add_f32"), ("v_fmac_f32", "v_fma_f32"),
           ("v_rcp", "v_rcp_f64"), ("v_rsq", "v_rcp_f64"), ("v_sqrt", "v_rcp_f64"), ("v_trunc", "v_add_f32"),
           ("v_lshl_add_u64", "v_mad_u64_u32"), ("v_mad_u64", "v_mad_u64_u32")]
    for p, row in fam:
        if base.startswith(p) and row in rates:
            return rates[row], row
    return None, None


def main():
    so = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(HERE), "cpu-raytracing-rt_amd",
                                                            "build", "librt_amd.so")
    rates = measured()
    res = {"source": "static opcode counts of each instance's code (llvm-objdump), priced with "
                     "profiles/r04/valu_rates_full.log (8 waves/SIMD, wall-clock cycles per wave64 instruction)",
           "rates": rates, "instances": {}}
    for co in code_objects(so):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", "--demangle", f.name],
                                 capture_output=True, text=True).stdout
        blocks = re.split(r"\n(?=[0-9a-f]+ <)", dis)
        for name, pat in INSTANCES.items():
            body = next((b for b in blocks if pat in b.split("\n", 1)[0]), None)
            if body is None:
                continue
            ops = Counter()
            for line in body.split("\n")[1:]:
                m = re.match(r"\s+(v_\S+)", line)
                if m:
                    ops[m.group(1)] += 1
            cls = {}
            for op, n in ops.items():
                k = class_of(op)
                c, _ = price(op, rates)
                e = cls.setdefault(k, {"static_count": 0, "priced": 0, "cycles": 0.0, "unpriced": {}, "top": Counter()})
                e["static_count"] += n
                e["top"][op] += n
                if c is None:
                    e["unpriced"][op] = n
                else:
                    e["priced"] += n
                    e["cycles"] += n * c
            out = {}
            for k, e in cls.items():
                out[k] = {"static_count": e["static_count"], "mean_cycles": e["cycles"] / max(e["priced"], 1),
                          "top": dict(e["top"].most_common(8)), "unpriced": e["unpriced"]}
            res["instances"][name] = {"kernel": pat, "classes": out}
    json.dump(res, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
