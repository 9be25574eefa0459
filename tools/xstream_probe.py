#!/usr/bin/env python3
"""Cost of a cross-stream dependency (measurement aid, profiles/r05/ab_runs.txt block 16):

    python tools/xstream_probe.py

A chain of N small kernels alternating between two streams, each link an event record on one
stream and a wait on the other, against the same chain on one stream; once with the default
(null) stream as one of the pair and once with two created streams.
"""
import time

import torch


def chain(sa, sb, n, x, cross):
    ev = [torch.cuda.Event() for _ in range(n)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        s = sa if (not cross or i % 2 == 0) else sb
        if cross and i > 0:
            s.wait_event(ev[i - 1])
        with torch.cuda.stream(s):
            x.add_(1.0)
        ev[i].record(s)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e6


def main():
    x = torch.zeros(1 << 20, device="cuda")
    d = torch.cuda.current_stream()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for _ in range(2):
        res = {
            "same_stream_us": round(chain(s1, s1, 200, x, False), 1),
            "created_pair_us": round(chain(s1, s2, 200, x, True), 1),
            "default_and_created_us": round(chain(d, s2, 200, x, True), 1),
        }
    print(res)


if __name__ == "__main__":
    main()
