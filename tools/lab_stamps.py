#!/usr/bin/env python3
"""Summarise tools/enc_lab stamp files: python3 tools/lab_stamps.py gpurun_out/lab_stamps_<v>.csv ..."""
import csv
import statistics as st
import sys
from collections import Counter

for fn in sys.argv[1:]:
    rows = list(csv.DictReader(open(fn)))
    t0 = min(int(r["start"]) for r in rows)
    S = [((int(r["start"]) - t0) / 100, (int(r["first"]) - t0) / 100, (int(r["last"]) - t0) / 100,
          (int(r["end"]) - t0) / 100, int(r["xcc"]), int(r["hwid"]), int(r["block"])) for r in rows]
    end = max(s[3] for s in S)
    print(fn, "tiles", len(S), "kernel span us %.1f" % end)
    for name, f in (("tile dur", lambda s: s[3] - s[0]), ("start->first wait", lambda s: s[1] - s[0]),
                    ("first->last step", lambda s: s[2] - s[1]), ("last step->end", lambda s: s[3] - s[2])):
        d = [f(s) for s in S]
        print("  %-18s us: min %.2f med %.2f max %.2f" % (name, min(d), st.median(d), max(d)))
    cu = Counter((s[4], s[5]) for s in S)
    print("  distinct (xcc,hwid)", len(cu), " block%8 != xcc:", sum(1 for s in S if s[6] % 8 != s[4]))
    B = 10
    n = int(end // B) + 1
    hs, he = Counter(int(s[0] // B) for s in S), Counter(int(s[3] // B) for s in S)
    print("  starts per %dus:" % B, [hs[i] for i in range(n)])
    print("  ends   per %dus:" % B, [he[i] for i in range(n)])
    # concurrent tiles over time
    conc = []
    for i in range(n):
        t = i * B + B / 2
        conc.append(sum(1 for s in S if s[0] <= t < s[3]))
    print("  resident tiles:  ", conc)
