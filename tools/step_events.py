#!/usr/bin/env python3
"""Measurement only: does recording HIP events between the kernels of a step cost time?

Times K headline steps (encode + decode_batch_out, k=200 m=32 B=1400, 8192 groups, e=32) by host
wall clock around a synchronized loop, in three forms, interleaved over several rounds:
  none    no events at all
  lib     the library's stage events only (cauchy_256_profile: 4 per decode)
  bench   bench.py's form: 3 torch events per step + the library's stage events

    python tools/step_events.py [--steps 20] [--rounds 3]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--rounds", type=int, default=3)
    a = p.parse_args()
    import torch
    import shorthair_amd as sh
    k, m, B, G = 200, 32, 1400, 8192
    sh.cauchy_256_init()
    data = torch.empty((G, k, B), dtype=torch.uint8, device="cuda")
    rec = torch.empty((G, m, B), dtype=torch.uint8, device="cuda")
    sh.fill_synthetic(data, k, B, G, 0, 0xBE)
    sh.encode_batch(k, m, B, G, data, rec)
    rows = np.zeros((G, k), np.uint8)
    for g in range(G):
        _, rows[g] = sh.erasure_pattern(g, k, m, 0xBE, m)
    d_rows = torch.from_numpy(rows).cuda()
    whole = torch.cat([data, rec], dim=1)
    blocks = whole[torch.arange(G, device="cuda")[:, None], d_rows.long()].contiguous()
    del whole
    out = torch.empty((G, m, B), dtype=torch.uint8, device="cuda")
    orow = torch.empty((G, m), dtype=torch.uint8, device="cuda")
    ocnt = torch.empty(G, dtype=torch.int32, device="cuda")
    sh.batch_reserve(k, m, B, G)
    stream = torch.cuda.current_stream()

    def run(form):
        evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(a.steps)]
        sh.profile(a.steps if form != "none" else 0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.steps):
            if form == "bench":
                evs[i][0].record(stream)
            sh.encode_batch(k, m, B, G, data, rec)
            if form == "bench":
                evs[i][1].record(stream)
            sh.decode_batch_out(k, m, B, G, blocks, d_rows, out, orow, ocnt)
            if form == "bench":
                evs[i][2].record(stream)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps * 1e3
        sh.profile(0)
        return dt

    for _ in range(2):
        run("none")
    res = {f: [] for f in ("none", "lib", "bench")}
    for _ in range(a.rounds):
        for f in res:
            res[f].append(run(f))
    gib = 2 * G * (k + m) * B / 2**30
    for f, v in res.items():
        print(f"{f:6s} ms/step " + " ".join(f"{x:.4f}" for x in v) + f"   median {np.median(v):.4f}"
              f"  -> {gib / (np.median(v) * 1e-3):.1f} GiB/s")


if __name__ == "__main__":
    main()
