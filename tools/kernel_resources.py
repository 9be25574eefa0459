#!/usr/bin/env python3
"""Per-kernel register / scratch / LDS usage of the gfx950 code objects inside a built library.

    python tools/kernel_resources.py shorthair_amd/libcauchy256.so [NAME_SUBSTRING]

Finds every clang offload bundle in the file (the .hip_fatbin data), extracts its gfx950 code
objects and prints the AMDGPU metadata of each kernel (llvm-readelf --notes). Measurement aid only.
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"


def code_objects(blob):
    pos = 0
    while True:
        i = blob.find(MAGIC, pos)
        if i < 0:
            return
        n = struct.unpack_from("<Q", blob, i + 24)[0]
        off = i + 32
        for _ in range(n):
            o, size, tlen = struct.unpack_from("<QQQ", blob, off)
            triple = blob[off + 24:off + 24 + tlen].decode()
            off += 24 + tlen
            if "gfx950" in triple and size:
                yield blob[i + o:i + o + size]
        pos = i + 1


def main():
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    blob = open(path, "rb").read()
    seen = set()
    for co in code_objects(blob):
        with tempfile.NamedTemporaryFile(suffix=".co", delete=False) as f:
            f.write(co)
            name = f.name
        try:
            txt = subprocess.run([READELF, "--notes", name], capture_output=True, text=True).stdout
        finally:
            os.unlink(name)
        for blk in txt.split("  - .agpr_count")[1:]:
            get = lambda key: (re.search(r"\.%s:\s+(\S+)" % key, blk) or [None, "?"])[1]
            nm = get("name")
            if sub not in nm or nm in seen:
                continue
            seen.add(nm)
            print(f"{nm[:90]:90s} vgpr={get('vgpr_count')} agpr={blk.split()[1] if blk.split() else '?'} "
                  f"sgpr={get('sgpr_count')} scratch={get('private_segment_fixed_size')} "
                  f"lds={get('group_segment_fixed_size')} wg={get('max_flat_workgroup_size')}")


if __name__ == "__main__":
    main()
