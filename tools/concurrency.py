#!/usr/bin/env python3
"""Experiment: encode batch and decode batch of one bench step serial on one stream vs. forked
onto two streams (independent ops; does a stage-B / encode overlap raise whole-step throughput?)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")))


def main():
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
        _, rows[g] = sh.erasure_pattern(g, k, m, 0xBE, 32)
    d_rows = torch.from_numpy(rows).cuda()
    whole = torch.cat([data, rec], dim=1)
    blocks = whole[torch.arange(G, device="cuda")[:, None], d_rows.long()].contiguous()
    del whole
    out = torch.empty((G, 32, B), dtype=torch.uint8, device="cuda")
    orow = torch.empty((G, 32), dtype=torch.uint8, device="cuda")
    ocnt = torch.empty(G, dtype=torch.int32, device="cuda")
    sh.batch_reserve(k, m, B, G)
    s1 = torch.cuda.current_stream()
    s2 = torch.cuda.Stream()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fork = torch.cuda.Event()
    join = torch.cuda.Event()
    for mode in ("serial", "forked", "serial", "forked"):
        ts = []
        for it in range(12):
            ev[0].record(s1)
            sh.encode_batch(k, m, B, G, data, rec, s1.cuda_stream)
            if mode == "serial":
                sh.decode_batch_out(k, m, B, G, blocks, d_rows, out, orow, ocnt, s1.cuda_stream)
            else:
                fork.record(s1)
                s2.wait_event(fork)
                sh.decode_batch_out(k, m, B, G, blocks, d_rows, out, orow, ocnt, s2.cuda_stream)
                join.record(s2)
                s1.wait_event(join)
            ev[1].record(s1)
            torch.cuda.synchronize()
            if it >= 2:
                ts.append(ev[0].elapsed_time(ev[1]))
        print(f"{mode}: step {np.mean(ts):.3f} ms (min {np.min(ts):.3f})", flush=True)


if __name__ == "__main__":
    main()
