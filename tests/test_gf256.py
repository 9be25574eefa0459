"""CPU tests of the host-side gf256.h ABI (SURVEY §8a X1/X2, §8b gf256.o exports) exported by
libcauchy256.so: GF(2^8) with polynomial 0x14D, the reference's table conventions and its
GF256Ctx layout.

Pinned two ways: (1) against the REFERENCE gf256.cpp compiled in place (oracle/_ref, see
oracle/Makefile) -- the whole GF256Ctx table object byte for byte after both inits, and every
bulk helper on random unaligned spans, also before init (the reference's zero-table behaviour);
(2) against an independent restatement here (carry-less multiply mod 0x14D). The reference
comparison runs in a child process so the reference's gf256_init_ does not change the state of
the reference codec other tests (and bench.py's CPU baseline, "as shipped") load."""
import ctypes
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
REF = os.path.join(ROOT, "oracle", "_ref", "libref_cauchy.so")
CTX_BYTES = 157728

CHILD = r"""
import ctypes, json, random, sys
sys.path.insert(0, sys.argv[1])
import shorthair_amd
ours = shorthair_amd.lib
ref = ctypes.CDLL(sys.argv[2])
N = 157728
out = {}

def bind(lib):
    v, c, i, u8 = ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_uint8
    lib.gf256_init_.argtypes = [i]
    lib.gf256_add_mem.argtypes = [v, v, i]
    lib.gf256_add2_mem.argtypes = [v, v, v, i]
    lib.gf256_addset_mem.argtypes = [v, v, v, i]
    lib.gf256_mul_mem.argtypes = [v, v, u8, i]
    lib.gf256_muladd_mem.argtypes = [v, u8, v, i]
    lib.gf256_memswap.argtypes = [v, v, i]
for lib in (ours, ref):
    bind(lib)

def run_ops(lib, seed, cases):
    rnd = random.Random(seed)
    res = []
    for _ in range(cases):
        n = rnd.choice([0, 1, 3, 7, 15, 16, 17, 31, 32, 33, 63, 64, 100, 175, 255, 256, 1000, 1399])
        oz, ox, oy = rnd.randrange(8), rnd.randrange(8), rnd.randrange(8)
        y = rnd.choice([0, 1, 2, 3, 0x8e, 0xff, rnd.randrange(256)])
        z0 = bytes(rnd.randrange(256) for _ in range(n + 8))
        x0 = bytes(rnd.randrange(256) for _ in range(n + 8))
        w0 = bytes(rnd.randrange(256) for _ in range(n + 8))
        row = []
        for op in range(7):
            z = ctypes.create_string_buffer(z0, n + 8)
            x = ctypes.create_string_buffer(x0, n + 8)
            w = ctypes.create_string_buffer(w0, n + 8)
            pz, px, pw = (ctypes.addressof(b) for b in (z, x, w))
            if op == 0: lib.gf256_add_mem(pz + oz, px + ox, n)
            elif op == 1: lib.gf256_add2_mem(pz + oz, px + ox, pw + oy, n)
            elif op == 2: lib.gf256_addset_mem(pz + oz, px + ox, pw + oy, n)
            elif op == 3: lib.gf256_mul_mem(pz + oz, px + ox, y, n)
            elif op == 4: lib.gf256_muladd_mem(pz + oz, y, px + ox, n)
            elif op == 5: lib.gf256_memswap(pz + oz, px + ox, n)
            else: lib.gf256_mul_mem(pz + oz, pz + oz, y, n)  # in place
            row.append((z.raw + x.raw).hex())
        res.append(row)
    return res

# before init: the tables are zero in both (mul by y >= 2 gives zeros, y <= 1 still works)
out["pre_equal"] = run_ops(ours, 1, 40) == run_ops(ref, 1, 40)
out["init"] = [ours.gf256_init_(2), ref.gf256_init_(2), ours.gf256_init_(2), ours.gf256_init_(3)]
a = bytes((ctypes.c_uint8 * N).in_dll(ours, "GF256Ctx"))
b = bytes((ctypes.c_uint8 * N).in_dll(ref, "GF256Ctx"))
out["ctx_equal"] = a == b
out["ctx_first_diff"] = next((i for i in range(N) if a[i] != b[i]), -1)
out["post_equal"] = run_ops(ours, 2, 300) == run_ops(ref, 2, 300)
print(json.dumps(out))
"""


def _symbol_size(lib_path, name):
    out = subprocess.run(["nm", "-DS", "--defined-only", lib_path], capture_output=True, text=True,
                         check=True).stdout
    for line in out.splitlines():
        f = line.split()
        if f[-1] == name:
            return int(f[1], 16)
    return None


def test_ctx_layout_and_export():
    import shorthair_amd
    assert _symbol_size(shorthair_amd.LIB_PATH, "GF256Ctx") == CTX_BYTES
    if os.path.exists(REF):
        assert _symbol_size(REF, "GF256Ctx") == CTX_BYTES


def test_matches_reference_build():
    if not os.path.exists(REF):
        pytest.skip("oracle/_ref not built")
    p = subprocess.run([sys.executable, "-c", CHILD, ROOT, REF], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["init"] == [0, 0, 0, -1]
    assert r["pre_equal"]
    assert r["ctx_equal"], f"GF256Ctx differs from byte {r['ctx_first_diff']}"
    assert r["post_equal"]


def _clmul_mod(a, b, poly=0x14D):
    r = 0
    while b:
        if b & 1:
            r ^= a
        b >>= 1
        a <<= 1
        if a & 0x100:
            a ^= poly
    return r


def test_field_restatement():
    """Independent of the reference: MUL/DIV/INV/SQR are GF(2^8) mod 0x14D."""
    import shorthair_amd
    lib = shorthair_amd.lib
    lib.gf256_init_.argtypes = [ctypes.c_int]
    assert lib.gf256_init_(2) == 0 and lib.gf256_init_(1) == -1
    ctx = bytes((ctypes.c_uint8 * CTX_BYTES).in_dll(lib, "GF256Ctx"))
    mul = ctx[24576:24576 + 65536]
    div = ctx[24576 + 65536:24576 + 131072]
    inv = ctx[24576 + 131072:24576 + 131072 + 256]
    sqr = ctx[24576 + 131072 + 256:24576 + 131072 + 512]
    poly = int.from_bytes(ctx[CTX_BYTES - 28:CTX_BYTES - 24], "little")
    assert poly == 0x14D
    for y in range(0, 256, 7):
        for x in range(256):
            assert mul[(y << 8) | x] == _clmul_mod(x, y)
            if y:
                assert _clmul_mod(div[(y << 8) | x], y) == x
    for x in range(1, 256):
        assert _clmul_mod(inv[x], x) == 1 and sqr[x] == _clmul_mod(x, x)
    # bulk mul_mem against the restatement, unaligned and with a tail
    buf = (ctypes.c_uint8 * 301)(*[(i * 37 + 11) & 255 for i in range(301)])
    out = (ctypes.c_uint8 * 301)()
    lib.gf256_mul_mem.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint8, ctypes.c_int]
    lib.gf256_mul_mem(ctypes.addressof(out) + 1, ctypes.addressof(buf) + 3, 0xC3, 297)
    assert [out[1 + i] for i in range(297)] == [_clmul_mod(buf[3 + i], 0xC3) for i in range(297)]


def test_c_caller_of_gf256_runs_on_cpu(tmp_path):
    """A plain-C program written against include/gf256.h (the reference's gf256.h interface:
    gf256_init(), inline gf256_mul/div/inv, gf256_div_mem) links against libcauchy256.so and runs
    here: these helpers are host code and need no GPU."""
    import shorthair_amd
    src = tmp_path / "gf.c"
    src.write_text(r'''
#include "gf256.h"
#include <stdio.h>
int main(void) {
    if (gf256_init() != 0) return 2;
    unsigned char x[40], z[40], back[40];
    for (int i = 0; i < 40; ++i) x[i] = (unsigned char)(i * 29 + 7);
    gf256_mul_mem(z, x, 0x53, 40);
    gf256_div_mem(back, z, 0x53, 40);
    for (int i = 0; i < 40; ++i)
        if (back[i] != x[i] || z[i] != gf256_mul(x[i], 0x53)) return 3;
    if (gf256_mul(gf256_inv(0x53), 0x53) != 1 || gf256_div(gf256_sqr(9), 9) != 9) return 4;
    gf256_muladd_mem(z, 0x53, x, 40);  /* z ^= x * 0x53 -> 0 */
    for (int i = 0; i < 40; ++i)
        if (z[i]) return 5;
    printf("ok %u\n", GF256Ctx.Polynomial);
    return 0;
}
''')
    exe = tmp_path / "gf"
    inc = os.path.join(ROOT, "include")
    libdir = os.path.dirname(shorthair_amd.LIB_PATH)
    subprocess.run(["gcc", "-std=c99", "-O2", "-Wall", "-Werror", f"-I{inc}", str(src), "-o", str(exe),
                    f"-L{libdir}", "-lcauchy256", f"-Wl,-rpath,{libdir}"], check=True)
    res = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert res.returncode == 0 and "ok 333" in res.stdout, (res.returncode, res.stdout, res.stderr)
