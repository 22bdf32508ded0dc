"""Disassemble the gfx950 code object of a built .so/.o: python tools/disasm.py lib.so out.s"""
import subprocess
import sys
import tempfile

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from kstats import code_objects  # noqa: E402

if __name__ == "__main__":
    cos = list(code_objects(sys.argv[1]))
    with open(sys.argv[2], "w") as out:
        for co in cos:
            with tempfile.NamedTemporaryFile(suffix=".co") as f:
                f.write(co)
                f.flush()
                out.write(subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "-d", "--mcpu=gfx950", f.name],
                                         capture_output=True, text=True).stdout)
