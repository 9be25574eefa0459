#!/usr/bin/env python3
"""Print the headline ops and the sweep of a bench.py JSON line, and check it against an earlier
line (measurement aid):

    python tools/sweep_table.py gpurun_out/bench.log
    python tools/sweep_table.py new.json --against profiles/r04/f_bench_full.json [--tol 0.05]

With --against, every sweep row present in both lines (same config, k, m, B, groups, path) is
compared on encode_ms and decode_ms (and the headline's per-op times); a row more than --tol
(fraction, default 0.05) slower is listed as a regression and the exit status is 1. Box-to-box
spread of one library is about 5 %, so a flagged row is a prompt to rerun on
one box, not a verdict.
"""
import argparse
import json
import sys


def load(path):
    """The last bench JSON line of a file (a bench log, a .json or a .jsonl)."""
    last = None
    for line in open(path):
        line = line.strip()
        if line.startswith("{"):
            try:
                d = json.loads(line)
            except ValueError:
                continue
            if "sweep" in d or "ops" in d:
                last = d
    if last is None:
        raise SystemExit(f"{path}: no bench JSON line")
    return last


def row_key(s):
    return (s["config"], s["k"], s["m"], s["B"], s["groups"], s.get("path", ""))


def print_table(d):
    print(d["value"], d["unit"], d.get("ops"))
    for s in d.get("sweep", []):
        print(f"{s['config']:12s} ({s['k']},{s['m']},{s['B']}) {s['path']:6s} G={s['groups']:6d} "
              f"enc {s.get('encode_ms') or 0:7.4f} ms {s.get('encode_frac') or 0:6.4f}  "
              f"dec {s['decode_ms']:7.4f} ms {s['decode_frac']:6.4f}  e={s['mean_e']}  "
              f"product rate enc {s.get('encode_product_rate', 0)} dec {s.get('decode_product_rate', 0)}")


def compare(new, old, tol):
    """[(name, old_ms, new_ms, ratio)] for every timing more than tol slower in `new`."""
    out = []
    pairs = []
    a, b = old.get("ops") or {}, new.get("ops") or {}
    for f in ("encode_ms", "decode_ms", "decode_stageA_ms", "decode_stageB_ms"):
        if a.get(f) and b.get(f):
            pairs.append((f"headline {f}", a[f], b[f]))
    olds = {row_key(s): s for s in old.get("sweep", [])}
    for s in new.get("sweep", []):
        o = olds.get(row_key(s))
        if o is None:
            continue
        name = "{} ({},{},{}) G={} {}".format(*row_key(s))
        for f in ("encode_ms", "decode_ms"):
            if o.get(f) and s.get(f):
                pairs.append((f"{name} {f[:6]}", o[f], s[f]))
    for name, a, b in pairs:
        if b > a * (1.0 + tol):
            out.append((name, a, b, b / a))
    return out, len(pairs)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("line")
    ap.add_argument("--against", default=None)
    ap.add_argument("--tol", type=float, default=0.05)
    args = ap.parse_args(argv)
    new = load(args.line)
    print_table(new)
    if args.against is None:
        return 0
    regs, n = compare(new, load(args.against), args.tol)
    print(f"\n{n} timings compared against {args.against} (tolerance {args.tol:.0%})")
    for name, a, b, r in regs:
        print(f"REGRESSION {name}: {a:.4f} -> {b:.4f} ms ({r:.3f}x)")
    if not regs:
        print("no regression")
    return 1 if regs else 0


if __name__ == "__main__":
    sys.exit(main())
