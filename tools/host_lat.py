#!/usr/bin/env python3
"""Where the single-group ABI's time goes (measurement aid for DESIGN.md §5.1):

    python tools/host_lat.py [--calls 200]

Times, per call, at k=200 m=32 B=1400 e=32: cauchy_256_encode / cauchy_256_decode as bench.py's
host_path does; the host gather of the 200 caller blocks into pinned memory alone; an H2D copy of
those bytes from pinned memory (with its synchronize); a D2H of the 32 recovered blocks; and an
empty-kernel round trip (launch + synchronize). Run under rocprofv3 --kernel-trace --stats for
the kernels' own durations.
"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")))


def per_call(fn, n):
    fn()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    return (time.perf_counter() - t0) / n * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=200)
    args = ap.parse_args()
    import torch
    import shorthair_amd as sh
    assert sh.lib.cauchy_256_batch_init(0) == 0
    k, m, B, n = 200, 32, 1400, args.calls
    rng = np.random.default_rng(7)
    data = rng.integers(0, 256, size=(k, B), dtype=np.uint8)
    blocks = [data[x].copy() for x in range(k)]
    rec = np.empty((m, B), np.uint8)
    ptrs = [b.ctypes.data for b in blocks]
    res = {}
    res["encode_us"] = per_call(lambda: sh.cauchy_256_encode(k, m, ptrs, rec.ctypes.data, B), n)
    whole = np.concatenate([data, rec])
    rows = list(range(m, k)) + list(range(k, k + m))
    sets = []
    for _ in range(n + 1):
        bufs = [whole[r].copy() for r in rows]
        sets.append((bufs, (sh.Block * k)(*[sh.Block(b.ctypes.data, r) for b, r in zip(bufs, rows)])))
    it = iter(sets)
    res["decode_us"] = per_call(lambda: sh.cauchy_256_decode(k, m, next(it)[1], B), n)
    assert all(np.array_equal(sets[-1][0][k - m + i], data[i]) for i in range(m))
    pin = torch.empty(k * B + 256, dtype=torch.uint8).pin_memory()
    pv = pin.numpy()

    def gather():
        for x in range(k):
            ctypes.memmove(pv.ctypes.data + x * B, ptrs[x], B)
    res["host_gather_us"] = per_call(gather, n)
    dev = torch.empty(k * B + 256, dtype=torch.uint8, device="cuda")
    s = torch.cuda.Stream()

    def h2d():
        with torch.cuda.stream(s):
            dev.copy_(pin, non_blocking=True)
        s.synchronize()
    res["h2d_sync_us"] = per_call(h2d, n)
    outp = torch.empty(m * B, dtype=torch.uint8).pin_memory()

    def d2h():
        with torch.cuda.stream(s):
            outp.copy_(dev[: m * B], non_blocking=True)
        s.synchronize()
    res["d2h_sync_us"] = per_call(d2h, n)
    tiny = torch.empty(1, device="cuda")

    def kern():
        with torch.cuda.stream(s):
            tiny.add_(1)
        s.synchronize()
    res["empty_kernel_sync_us"] = per_call(kern, n)
    print({kk: round(v, 1) for kk, v in res.items()})


if __name__ == "__main__":
    main()
