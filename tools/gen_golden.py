#!/usr/bin/env python3
"""Generate tests/golden/ from the REAL reference codec (oracle/_ref/libref_cauchy.so).

The reference's own tests pin no codec results, so parity is pinned here: every
expected output below comes from catid/shorthair's cauchy_256.cpp/gf256.cpp compiled from
/root/reference by oracle/Makefile. Inputs are the synthetic PCG32 workload of
oracle/cauchy_oracle.c (ora_fill_block / ora_erasure_pattern); the SHA-256 of every input is
stored too, which pins the generator.

Outputs:
  tests/golden/golden_small.npz  full input/output vectors for every reference code path
  tests/golden/manifest.json     case list + SHA-256 digests (also for the large shapes)
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, ROOT)
from oracle import pyoracle as po  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")
CFG = 0x5348  # workload id for golden inputs


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    po.build()
    ref = po.reference()
    if ref is None:
        sys.exit("reference not built: needs /root/reference (run in the build container)")
    os.makedirs(OUT, exist_ok=True)
    arrays, cases = {}, []

    def enc_case(name, g, k, m, B, full=True, note=""):
        data = po.fill_group(g, k, B, CFG)
        rc, out = ref.encode(k, m, data, B)
        c = dict(kind="encode", name=name, g=g, k=k, m=m, B=B, cfg=CFG, rc=rc,
                 in_sha=sha(data), out_sha=sha(out), note=note, full=full)
        if full:
            arrays[name + "_out"] = out
        cases.append(c)
        return data, out, rc

    def dec_case(name, g, k, m, B, e_fixed, order="sorted", full=True, note=""):
        data = po.fill_group(g, k, B, CFG)
        rc_e, rec = ref.encode(k, m, data, B)
        assert rc_e == 0 or k + m > 256
        whole = np.concatenate([data, rec])
        if order == "all_original":
            rows = np.arange(k, dtype=np.uint8)
        else:
            _, rows = po.erasure_pattern(g, k, m, CFG, e_fixed)
            if order == "reversed":
                rows = rows[::-1].copy()
            elif order == "shuffled":
                rng = np.random.default_rng(g * 7919 + k)
                rows = rows[rng.permutation(k)].copy()
        blocks = [whole[r].copy() for r in rows]
        rc, new_rows = ref.decode(k, m, blocks, [int(r) for r in rows], B)
        outd = np.stack(blocks) if blocks else np.zeros((0, B), np.uint8)
        c = dict(kind="decode", name=name, g=g, k=k, m=m, B=B, cfg=CFG, e_fixed=e_fixed,
                 order=order, rc=rc, rows_in=[int(r) for r in rows], rows_out=new_rows,
                 in_sha=sha(np.stack([whole[r] for r in rows])), out_sha=sha(outd), note=note,
                 full=full)
        if full:
            arrays[name + "_out"] = outd
        cases.append(c)

    # ---- encode: every reference code path (cauchy_256.cpp:1479-1578) ----
    enc_case("enc_k1_copy", 1, 1, 4, 16, note="k<=1: data[0] copied to every output (:1485)")
    enc_case("enc_m1_xor", 2, 10, 1, 64, note="m==1: XOR of inputs only (:1503)")
    enc_case("enc_m1_odd_bytes", 3, 10, 1, 13, note="m==1 skips the B%8 check")
    enc_case("enc_m2", 4, 12, 2, 40, note="static table m=2, non-window path (:1538)")
    enc_case("enc_m3", 5, 10, 3, 64)
    enc_case("enc_m4_1400", 6, 30, 4, 1400)
    enc_case("enc_m5_window", 7, 12, 5, 40, note="m>4 window path, static table m=5 (:1534)")
    enc_case("enc_m6_window", 8, 20, 6, 48)
    enc_case("enc_m7_generated", 9, 20, 7, 48, note="m>=7 generated matrix (:453)")
    enc_case("enc_m9", 10, 20, 9, 48)
    enc_case("enc_k64_m16_1400", 11, 64, 16, 1400, note="C2 shape, one group")
    enc_case("enc_k200_m32_1400", 12, 200, 32, 1400, note="headline shape, one group")
    enc_case("enc_k250_m6_8", 13, 250, 6, 8)
    enc_case("enc_k128_m128_8", 14, 128, 128, 8)
    enc_case("enc_k3_m253_8", 15, 3, 253, 8)
    enc_case("enc_k2_m2_8", 16, 2, 2, 8)
    enc_case("enc_k224_m32_256", 17, 224, 32, 256)
    enc_case("enc_k28_m4_256", 18, 28, 4, 256)
    enc_case("enc_bad_km", 19, 200, 60, 16, note="k+m>256: rc=-1 AFTER row 0 written (:1509)")
    enc_case("enc_bad_bytes", 20, 20, 4, 12, note="B%8!=0: rc=-1 after row 0 written")

    # ---- decode: every path (cauchy_256.cpp:1233-1392) ----
    dec_case("dec_k1", 30, 1, 3, 16, 1, note="k<=1: blocks[0].row=0 (:1236)")
    dec_case("dec_m1", 31, 10, 1, 64, 1, order="shuffled", note="m==1: row stays >= k (:487)")
    dec_case("dec_none_erased", 32, 20, 4, 64, 0, order="all_original", note="no erasures (:1266)")
    dec_case("dec_m2_e1", 33, 12, 2, 40, 1)
    dec_case("dec_m3_e3", 34, 12, 3, 24, 3, order="shuffled")
    dec_case("dec_m4_e4_1400", 35, 30, 4, 1400, 4, order="reversed", note="e<=4: plain GE")
    dec_case("dec_m6_e5", 36, 20, 6, 40, 5, order="shuffled", note="e>4: windowed GE")
    dec_case("dec_m9_e9", 37, 30, 9, 48, 9, order="shuffled")
    dec_case("dec_m12_e4", 38, 40, 12, 16, 4)
    dec_case("dec_m32_e20", 39, 25, 32, 16, 20, order="shuffled")
    dec_case("dec_k64_m16_e16_1400", 40, 64, 16, 1400, 16)
    dec_case("dec_k200_m32_e32_1400", 41, 200, 32, 1400, 32, note="headline shape, worst case")
    dec_case("dec_k200_m32_e7_1400", 42, 200, 32, 1400, 7, order="shuffled")
    dec_case("dec_k128_m128_e100_8", 43, 128, 128, 8, 100, order="shuffled")
    dec_case("dec_k3_m253_e3_8", 44, 3, 253, 8, 3)
    dec_case("dec_bad_km", 45, 200, 60, 16, 4, note="k+m>256: rc=-1 (:1271)")
    # e = m at the searched tables (m <= 6): every recovery row replaces an erasure
    dec_case("dec_m6_e6", 46, 20, 6, 40, 6, order="shuffled", note="m=6, e=6: 6x6 submatrix")
    dec_case("dec_m6_e6_1400", 47, 30, 6, 1400, 6, note="m=6, e=6 at B=1400")
    dec_case("dec_m5_e5", 48, 12, 5, 64, 5, order="reversed", note="m=5, e=5")

    # ---- config 1: the call shapes the reference's loopback Tester issues (SURVEY.md §3.4:
    # k=200/m=56/B=1352, k=190/m=66/B in {1336,1344}, decodes with 12-28 erasures). Tester.cpp
    # itself does not compile unmodified (Counter.h:306,309), so these are driven directly.
    enc_case("tester_enc_200_56_1352", 50, 200, 56, 1352)
    enc_case("tester_enc_190_66_1336", 51, 190, 66, 1336)
    enc_case("tester_enc_190_66_1344", 52, 190, 66, 1344)
    dec_case("tester_dec_200_56_1352_e12", 53, 200, 56, 1352, 12, order="shuffled")
    dec_case("tester_dec_200_56_1352_e28", 54, 200, 56, 1352, 28)
    dec_case("tester_dec_190_66_1336_e20", 55, 190, 66, 1336, 20, order="reversed")

    # ---- large shapes: digests only (regenerable inputs) ----
    for g in range(4):
        enc_case(f"big_enc_c2_g{g}", 1000 + g, 64, 16, 1400, full=False)
        enc_case(f"big_enc_c3_g{g}", 2000 + g, 200, 32, 1400, full=False)
        dec_case(f"big_dec_c3_e32_g{g}", 3000 + g, 200, 32, 1400, 32, full=False)
        dec_case(f"big_dec_c3_rand_g{g}", 4000 + g, 200, 32, 1400, 0, full=False)
    for (k, m) in [(28, 4), (112, 16), (224, 32)]:
        for B in (256, 1400, 65536):
            enc_case(f"big_enc_c4_{k}_{m}_{B}", 5000 + k + B, k, m, B, full=False)
            dec_case(f"big_dec_c4_{k}_{m}_{B}", 6000 + k + B, k, m, B, 0, full=False)

    # ---- off-grid shapes (no compile-time kernels: the runtime-coefficient tile kernels code
    # them): what Shorthair's policy issues between the compiled pairs (k = packets queued in the
    # interval, m = R clamped to 256 - k, Shorthair.cpp:1130-1174, :502-504), plus the edges of
    # the tile kernels (one part, 16 parts, two launches for m > 128, short sub-blocks).
    for i, (k, m, B, e) in enumerate([(120, 136, 1400, 64), (150, 40, 1400, 40), (50, 10, 1000, 7),
                                      (180, 76, 1352, 33), (2, 254, 128, 2), (100, 100, 200, 0),
                                      (5, 3, 128, 3), (70, 72, 520, 0)]):
        enc_case(f"offgrid_enc_{k}_{m}_{B}", 7000 + i, k, m, B, full=False)
        dec_case(f"offgrid_dec_{k}_{m}_{B}_e{e or 'r'}", 7100 + i, k, m, B, e, order="shuffled", full=False)

    np.savez_compressed(os.path.join(OUT, "golden_small.npz"), **arrays)
    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump(dict(generator="tools/gen_golden.py", source="oracle/_ref/libref_cauchy.so "
                       "(catid/shorthair cauchy_256.cpp + gf256.cpp)", cases=cases), f, indent=1)
    print(f"{len(cases)} cases, {len(arrays)} full vectors")


if __name__ == "__main__":
    main()
