#!/usr/bin/env python3
"""Per-wave cycle split from tools/enc_lab stamp files (rows variant / base with ST):
compute (between waits), own-DMA vmcnt wait, barrier wait -- mean over tiles, per wave index."""
import csv
import sys

for fn in sys.argv[1:]:
    rows = list(csv.DictReader(open(fn)))
    tot = [[0.0, 0.0, 0.0] for _ in range(8)]
    n = 0
    for r in rows:
        v = [int(x) for x in r["wavecyc"].split()]
        if len(v) < 24 or sum(v) == 0:
            continue
        n += 1
        for w in range(8):
            for j in range(3):
                tot[w][j] += v[3 * w + j]
    print(fn, "tiles", n)
    for w in range(8):
        c, d, b = (x / max(n, 1) for x in tot[w])
        s = c + d + b
        print("  wave %d: compute %7.0f  dma-wait %7.0f  barrier %7.0f cycles  (%.0f%% / %.0f%% / %.0f%%)" % (
            w, c, d, b, 100 * c / s, 100 * d / s, 100 * b / s))
