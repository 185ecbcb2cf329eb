"""Register, spill and scratch figures of every path/trace kernel instance in a
built librt_amd.so (reads the gfx950 code object's AMDGPU metadata notes).

    python tools/kernel_regs.py [path/to/librt_amd.so] [name-filter]
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def code_objects(so_path):
    """The gfx950 code objects of the .so's offload bundles (plain or compressed)."""
    data = open(so_path, "rb").read()
    out = []
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    pos = 0
    while True:
        i = data.find(magic, pos)
        if i < 0:
            break
        n = struct.unpack_from("<Q", data, i + 24)[0]
        p = i + 32
        for _ in range(n):
            off, size, idlen = struct.unpack_from("<QQQ", data, p)
            ident = data[p + 24:p + 24 + idlen].decode()
            p += 24 + idlen
            if "gfx950" in ident:
                out.append(data[i + off:i + off + size])
        pos = i + 24
    if not out and b"CCOB" in data:
        # compressed bundle: let the bundler decompress it
        with tempfile.TemporaryDirectory() as d:
            j = data.find(b"CCOB")
            src = os.path.join(d, "b.bin")
            open(src, "wb").write(data[j:])
            dst = os.path.join(d, "k.co")
            subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={src}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={dst}"], check=True)
            out.append(open(dst, "rb").read())
    return out


def main():
    so = sys.argv[1] if len(sys.argv) > 1 else "cpu-raytracing-rt_amd/build/librt_amd.so"
    filt = sys.argv[2] if len(sys.argv) > 2 else "_kernel"
    for co in code_objects(so):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            notes = subprocess.run([f"{LLVM}/llvm-readobj", "--notes", f.name], capture_output=True,
                                   text=True).stdout
            names = subprocess.run(["c++filt"], input="\n".join(
                re.findall(r"\.name:\s+(\S+)", notes)), capture_output=True, text=True).stdout.split("\n")
        blocks = re.split(r"\n\s+- \.agpr_count", notes)[1:]
        print(f"{'vgpr':>5} {'vspill':>6} {'sgpr':>5} {'sspill':>6} {'scratch':>7} {'lds':>6}  kernel")
        for blk, dn in zip(blocks, names):
            def g(k):
                m = re.search(r"\." + k + r":\s+(\S+)", blk)
                return m.group(1) if m else "?"
            if filt not in dn:
                continue
            print(f"{g('vgpr_count'):>5} {g('vgpr_spill_count'):>6} {g('sgpr_count'):>5} "
                  f"{g('sgpr_spill_count'):>6} {g('private_segment_fixed_size'):>7} "
                  f"{g('group_segment_fixed_size'):>6}  {dn[:150]}")


if __name__ == "__main__":
    main()
