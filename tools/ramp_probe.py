#!/usr/bin/env python3
"""Measurement only: how many headline steps does the GPU need, from idle, to reach its steady
step time? Sets up like bench.py, lets the GPU idle, then runs N steps with an event pair per step
and prints every step's time (the events' own cost is ~1 % of a step, the same for every step).

    python tools/ramp_probe.py [--steps 80] [--idle 1.0]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=80)
    p.add_argument("--idle", type=float, default=1.0, help="seconds of GPU idle before the steps")
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
    for _ in range(3):
        sh.encode_batch(k, m, B, G, data, rec)
        sh.decode_batch_out(k, m, B, G, blocks, d_rows, out, orow, ocnt)
    torch.cuda.synchronize()
    time.sleep(a.idle)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)]
    evs[0].record(stream)
    for i in range(a.steps):
        sh.encode_batch(k, m, B, G, data, rec)
        sh.decode_batch_out(k, m, B, G, blocks, d_rows, out, orow, ocnt)
        evs[i + 1].record(stream)
    torch.cuda.synchronize()
    ms = [evs[i].elapsed_time(evs[i + 1]) for i in range(a.steps)]
    print("per-step ms:", " ".join(f"{x:.3f}" for x in ms))
    for lo in range(0, a.steps, 10):
        print(f"steps {lo:3d}-{lo + 9:3d}: mean {np.mean(ms[lo:lo + 10]):.4f} ms")


if __name__ == "__main__":
    main()
