"""VGPR / SGPR / spill / scratch of the kernels in a built .so or .o (reads the gfx950 code object
out of the clang offload bundle and its AMDGPU metadata note).
usage: python tools/kstats.py lib.so [kernel-regex]"""
import re
import struct
import subprocess
import sys
import tempfile


def code_objects(path):
    data = open(path, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    pos = data.find(magic)
    while pos >= 0:
        n = struct.unpack_from("<Q", data, pos + 24)[0]
        p = pos + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tl].decode()
            p += 24 + tl
            if "gfx950" in triple and size:
                yield data[pos + off:pos + off + size]
        pos = data.find(magic, pos + 1)


def main():
    path = sys.argv[1]
    pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else r"ib_(cn|vn)_fast")
    for co in code_objects(path):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            txt = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", f.name],
                                 capture_output=True, text=True).stdout
        for blk in re.split(r"\n\s+- \.", txt):
            m = re.search(r"\.name:\s+(\S+)", blk)
            if not m or not pat.search(m.group(1)) or ".vgpr_count" not in blk:
                continue

            def g(k):
                r = re.search(r"\." + k + r":\s+(\S+)", blk)
                return r.group(1) if r else "?"
            print(f"{m.group(1)[:58]:58s} vgpr={g('vgpr_count'):>4} sgpr={g('sgpr_count'):>3} "
                  f"spill={g('vgpr_spill_count'):>3} scratch={g('private_segment_fixed_size')}")


if __name__ == "__main__":
    main()
