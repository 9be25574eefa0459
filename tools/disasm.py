#!/usr/bin/env python3
"""Disassemble the gfx950 code objects of a built object / library (measurement aid only).

    python tools/disasm.py shorthair_amd/build_obj/fixed_k200_m32_enc.hip.o > /tmp/enc.s
"""
import os
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kernel_resources import code_objects  # noqa: E402

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"

if __name__ == "__main__":
    blob = open(sys.argv[1], "rb").read()
    for co in code_objects(blob):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            sys.stdout.write(subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", f.name],
                                            capture_output=True, text=True).stdout)
