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
    p.add_argument("--concurrent", action="store_true", help="encode and decode on two streams at once")
    p.add_argument("--zero", action="store_true", help="all-zero data blocks (data-dependent power / DVFS check)")
    p.add_argument("--digest", action="store_true",
                   help="print SHA-256 digests of the recovery blocks and the decoded blocks (variant parity)")
    a = p.parse_args()
    import torch
    import shorthair_amd as sh
    k, m, B, G = a.k, a.m, a.block, a.groups
    sh.cauchy_256_init()
    data = torch.empty((G, k, B), dtype=torch.uint8, device="cuda")
    rec = torch.empty((G, m, B), dtype=torch.uint8, device="cuda")
    sh.fill_synthetic(data, k, B, G, 0, 0xBE)
    if a.zero:
        data.zero_()
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
    if a.concurrent:
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for it in range(a.iters + 1):
            if it == 1:
                torch.cuda.synchronize()
                e0.record()
            ev_s = torch.cuda.Event()
            ev_s.record()
            s1.wait_event(ev_s)
            s2.wait_event(ev_s)
            sh.encode_batch(k, m, B, G, data, rec, s1.cuda_stream)
            sh.decode_batch_out(k, m, B, G, blocks, d_rows, out, orow, ocnt, s2.cuda_stream)
            d1, d2 = torch.cuda.Event(), torch.cuda.Event()
            d1.record(s1)
            d2.record(s2)
            torch.cuda.current_stream().wait_event(d1)
            torch.cuda.current_stream().wait_event(d2)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        tot = G * (k + m) * B + G * (k + a.erasures) * B
        print(f"{os.path.basename(sh.LIB_PATH)} concurrent encode||decode: {ms:.3f} ms per step "
              f"({tot / ms / 1e6:.0f} GB/s, {tot / ms / 1e-3 / 2**30:.0f} GiB/s)")
        return
    sh.profile(a.iters)
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
    if a.digest:
        import hashlib
        torch.cuda.synchronize()
        dig = {"recovery": hashlib.sha256(rec.cpu().numpy().tobytes()).hexdigest()[:16]}
        if a.op in ("decode", "both"):
            # the decoded blocks must equal the erased originals (device round trip)
            lost = [[x for x in range(k) if x not in set(rows[g].tolist())] for g in range(min(G, 64))]
            ok = all(torch.equal(out[g, :len(l)].cpu(), data[g, l].cpu()) for g, l in enumerate(lost) if l)
            dig["decoded"] = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16]
            dig["roundtrip_ok"] = ok
        print("digest", dig)
    enc_b = G * (k + m) * B
    dec_b = G * (k + a.erasures) * B
    print(f"{os.path.basename(sh.LIB_PATH)} {a.op}: encode {te / a.iters:.3f} ms ({enc_b / (te / a.iters) / 1e9:.0f} GB/s)"
          f"  decode {td / a.iters:.3f} ms ({dec_b / (td / a.iters) / 1e9:.0f} GB/s)"
          + ("" if a.op == "encode" else "  stages setup/A/B ms: %s" % " / ".join(f"{x:.3f}" for x in (sh.profile_read() or ()))))


if __name__ == "__main__":
    main()
