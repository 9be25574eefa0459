#!/usr/bin/env python3
"""BASELINE config C1: capture real cauchy_256 encode/decode calls of the reference's protocol
layer and commit them as golden fixtures (tests/golden/c1_capture.npz).

oracle/_ref/shorthair_capture is the reference's unchanged Shorthair.cpp / PacketAllocator.cpp /
SiameseTools.cpp (compiled in place from /root/reference, oracle/Makefile) running the
Tester-shaped loopback of oracle/shorthair_link.cpp on the REFERENCE codec (_ref/libref_cauchy.so),
with every codec call recorded by oracle/capture_wrap.cpp (-Wl,--wrap). CPU only; run here:

    make -C oracle && python tools/capture_c1.py

The fixtures hold each call's real inputs -- Shorthair-framed, variable-length, misaligned packet
blocks (the pointer's address mod 16 is kept) -- and the reference codec's outputs.
"""
import glob
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
EXE = os.path.join(ROOT, "oracle", "_ref", "shorthair_capture")
OUT = os.path.join(ROOT, "tests", "golden", "c1_capture.npz")
KEEP_ENC, KEEP_DEC = (0, 2), (0, 1)  # (200,56,1352) and (190,66,1344) encodes; (200,56) and (190,66) decodes


def parse(path):
    b = open(path, "rb").read()
    k, m, B, rc = (int(x) for x in np.frombuffer(b[:16], np.int32))
    off = 16
    align = np.frombuffer(b[off:off + 4 * k], np.int32).astype(np.uint8)
    off += 4 * k
    rest = np.frombuffer(b[off:], np.uint8)
    return k, m, B, rc, align, rest


def main():
    if not os.path.exists(EXE):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    arrays = {}
    with tempfile.TemporaryDirectory() as d:
        env = dict(os.environ, CAPTURE_DIR=d, CAPTURE_MAX="4")
        r = subprocess.run([EXE, "--seconds", "1.5"], env=env, capture_output=True, text=True, timeout=120)
        print(r.stdout.strip())
        for n in KEEP_ENC:
            k, m, B, rc, align, rest = parse(os.path.join(d, f"{n}_enc.bin"))
            data = rest[:k * B].reshape(k, B)
            out = rest[k * B:k * B + m * B].reshape(m, B)
            p = f"enc{n}_"
            arrays.update({p + "kmbrc": np.array([k, m, B, rc], np.int32), p + "align": align,
                           p + "data": data, p + "out": out})
        for n in KEEP_DEC:
            k, m, B, rc, align, rest = parse(os.path.join(d, f"{n}_dec.bin"))
            rows0 = rest[:k]
            data0 = rest[k:k + k * B].reshape(k, B)
            rows1 = rest[k + k * B:2 * k + k * B]
            data1 = rest[2 * k + k * B:].reshape(k, B)
            changed = np.nonzero(rows0 >= k)[0]  # recovery blocks: they receive the recovered data
            assert np.array_equal(np.delete(data0, changed, axis=0), np.delete(data1, changed, axis=0))
            p = f"dec{n}_"
            arrays.update({p + "kmbrc": np.array([k, m, B, rc], np.int32), p + "align": align,
                           p + "rows_in": rows0, p + "data_in": data0, p + "rows_out": rows1,
                           p + "idx": changed.astype(np.int32), p + "data_out": data1[changed]})
    np.savez_compressed(OUT, **arrays)
    print("wrote", os.path.relpath(OUT, ROOT), os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    sys.exit(main())
