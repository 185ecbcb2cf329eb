"""Loops of one kernel in an llvm-objdump listing: each backward branch's address
range with its instruction count and the scratch / vector-memory / LDS ops inside.

    python tools/isa_loops.py listing.s [kernel-substring]
(listing: llvm-objdump -d --mcpu=gfx950 of the code object, tools/kernel_regs.py
extracts it)
"""
import re
import sys


def main():
    text = open(sys.argv[1]).read().split("\n")
    filt = sys.argv[2] if len(sys.argv) > 2 else None
    ins = []  # (offset, text)
    cur = None
    for line in text:
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
        if m:
            cur = m.group(1)
            continue
        if cur is None or (filt and filt not in cur):
            continue
        m = re.search(r"//\s*([0-9A-F]+):", line)
        if not m:
            continue
        ins.append((int(m.group(1), 16), line.strip()))
    if not ins:
        sys.exit("no instructions")
    base = ins[0][0]
    loops = []
    for off, t in ins:
        m = re.search(r"<\S+\+0x([0-9a-f]+)>", t)
        if m and ("branch" in t):
            tgt = base + int(m.group(1), 16) - (ins[0][0] - base)
            tgt = int(m.group(1), 16) + base
            if tgt <= off:
                loops.append((tgt, off))
    print(f"{len(ins)} instructions, scratch st {sum('scratch_store' in t for _, t in ins)} "
          f"ld {sum('scratch_load' in t for _, t in ins)}")
    for a, b in sorted(loops):
        body = [t for o, t in ins if a <= o <= b]
        def n(p):
            return sum(p in t for t in body)
        print(f"loop {a - base:#7x}-{b - base:#7x}: {len(body):5d} ins, scratch st {n('scratch_store'):3d} "
              f"ld {n('scratch_load'):3d}, vmem ld {n('global_load') + n('buffer_load'):3d} "
              f"st {n('global_store') + n('buffer_store'):3d}, lds {n('ds_'):3d}, s_waitcnt {n('s_waitcnt'):3d}")


if __name__ == "__main__":
    main()
