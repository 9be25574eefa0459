#!/usr/bin/env python3
"""Distribution of the 4-step ring intervals in tools/enc_lab stamp files (measurement only)."""
import csv
import sys

for fn in sys.argv[1:]:
    rows = list(csv.DictReader(open(fn)))
    W = [[int(x) for x in r["waits"].split()] for r in rows]
    allv = sorted((w[i + 1] - w[i]) / 100 for w in W for i in range(49) if w[i] >= 0 and w[i + 1] >= 0)
    n = len(allv)
    print("%s 4-step intervals us: p10 %.2f p50 %.2f p90 %.2f p99 %.2f max %.2f mean %.2f" % (
        fn, allv[n // 10], allv[n // 2], allv[9 * n // 10], allv[99 * n // 100], allv[-1], sum(allv) / n))
