#!/usr/bin/env python3
"""Run one codec op repeatedly on device-resident synthetic data (for rocprofv3 PMC passes).

    python tools/run_ops.py --op encode|decode|both --iters 5 [--k 200 --m 32 --block 1400 --groups 8192]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--op", default="both")
    p.add_argument("--iters", type=int, default=5)
    p.add_argument("--k", type=int, default=200)
    p.add_argument("--m", type=int, default=32)
    p.add_argument("--block", type=int, default=1400)
    p.add_argument("--groups", type=int, default=8192)
    p.add_argument("--erasures", type=int, default=32)
    a = p.parse_args()
    import torch
    import shorthair_amd as sh
    k, m, B, G = a.k, a.m, a.block, a.groups
    sh.cauchy_256_init()
    data = torch.empty((G, k, B), dtype=torch.uint8, device="cuda")
    rec = torch.empty((G, m, B), dtype=torch.uint8, device="cuda")
    sh.fill_synthetic(data, k, B, G, 0, 0xBE)
    sh.encode_batch(k, m, B, G, data, rec)
    if a.op in ("decode", "both"):
        rows = np.zeros((G, k), np.uint8)
        for g in range(G):
            _, rows[g] = sh.erasure_pattern(g, k, m, 0xBE, a.erasures)
        d_rows = torch.from_numpy(rows).cuda()
        whole = torch.cat([data, rec], dim=1)
        blocks = whole[torch.arange(G, device="cuda")[:, None], d_rows.long()].contiguous()
        del whole
        emax = min(k, m)
        out = torch.empty((G, emax, B), dtype=torch.uint8, device="cuda")
        orow = torch.empty((G, emax), dtype=torch.uint8, device="cuda")
        ocnt = torch.empty(G, dtype=torch.int32, device="cuda")
        sh.batch_reserve(k, m, B, G)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    te = td = 0.0
    for _ in range(a.iters):
        ev[0].record()
        if a.op in ("encode", "both"):
            sh.encode_batch(k, m, B, G, data, rec)
        ev[1].record()
        if a.op in ("decode", "both"):
            sh.decode_batch_out(k, m, B, G, blocks, d_rows, out, orow, ocnt)
        ev[2].record()
        torch.cuda.synchronize()
        te += ev[0].elapsed_time(ev[1])
        td += ev[1].elapsed_time(ev[2])
    enc_b = G * (k + m) * B
    dec_b = G * (k + a.erasures) * B
    print(f"{os.path.basename(sh.LIB_PATH)} {a.op}: encode {te / a.iters:.3f} ms ({enc_b / (te / a.iters) / 1e9:.0f} GB/s)"
          f"  decode {td / a.iters:.3f} ms ({dec_b / (td / a.iters) / 1e9:.0f} GB/s)")


if __name__ == "__main__":
    main()
