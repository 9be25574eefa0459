#!/usr/bin/env python3
"""Code-layout pass for the compile-time kernels (measurement build, round 5).

    python tools/il_reorder.py in.s out.s [--group G]

The kernels run P part-waves per workgroup, each through its OWN straight-line body (~0.5 MB of
code at (200, 32)): every workgroup fetches P separate instruction streams, and the part-waves
meet at a ring barrier every 4 steps, so a part stalled on an instruction line holds the others
(round 5: every part running part 0's code, one stream per workgroup, was 12 % faster). This pass
takes the device assembly of a kernel generated with SH_IL_MARK=1 (each unit of part p starts
with the comment ";shu p u", the body ends with ";shu p end"), cuts each part's body into its
units and lays them out interleaved -- unit u of parts 0..P-1 adjacent, then unit u+1 -- so the
part-waves of a workgroup walk one region of code: a wave's sequential instruction fetch past the
end of its chunk brings in the next part's chunk of the same unit. Each chunk ends in an
explicit s_branch to the same part's next chunk (a few KB away); the part's prologue reaches its
first chunk and the last chunk its epilogue with long branches (s_getpc / s_add / s_setpc through
s[44:45], the pair hipcc's own branch relaxation uses). Labels, the out-of-line blocks and every
branch between them move with their code; the assembler re-resolves them.

--group G: interleave G units per chunk (fewer branches, longer runs per part).
"""
import re
import sys


def main():
    args = sys.argv[1:]
    group = 1
    if "--group" in args:
        i = args.index("--group")
        group = int(args[i + 1])
        del args[i:i + 2]
    src, dst = args
    lines = open(src).read().split("\n")
    mark = re.compile(r"^\s*;shu (\d+) (\d+|end)\s*$")
    pos = {}  # (part, unit or 'end') -> line index of the marker comment
    for i, l in enumerate(lines):
        m = mark.match(l)
        if m:
            pos[(int(m.group(1)), m.group(2) if m.group(2) == "end" else int(m.group(2)))] = i
    parts = sorted({p for p, _ in pos})
    units = {p: sorted(u for q, u in pos if q == p and u != "end") for p in parts}
    U = len(units[parts[0]])
    assert all(units[p] == list(range(U)) for p in parts), "every part needs units 0..U-1"
    assert all((p, "end") in pos for p in parts)
    # the marker comment sits inside ;;#ASMSTART / ;;#ASMEND: cut right before the ASMSTART line
    def cut(i):
        return i - 1 if lines[i - 1].strip() == ";;#ASMSTART" else i

    starts = {(p, u): cut(pos[(p, u)]) for p in parts for u in range(U)}
    ends = {p: cut(pos[(p, "end")]) for p in parts}
    chunks = {}
    for p in parts:
        for g0 in range(0, U, group):
            a = starts[(p, g0)]
            b = starts[(p, g0 + group)] if g0 + group < U else ends[p]
            chunks[(p, g0)] = (a, b)
    # every part's body must be contiguous and disjoint from the others
    regions = sorted((starts[(p, 0)], ends[p], p) for p in parts)
    for (a0, b0, _), (a1, b1, _) in zip(regions, regions[1:]):
        assert b0 <= a1, "part bodies overlap"
    first = regions[0][2]  # the interleaved block replaces the first body in the file

    def lbl(p, g):
        return f".Lshu_{p}_{g}" if g < U else f".Lshu_{p}_end"

    def longbr(target, tag):
        return ["\ts_getpc_b64 s[44:45]",
                f".Lshu_pc_{tag}:",
                f"\ts_add_u32 s44, s44, ({target}-.Lshu_pc_{tag})&4294967295",
                f"\ts_addc_u32 s45, s45, ({target}-.Lshu_pc_{tag})>>32",
                "\ts_setpc_b64 s[44:45]"]

    inter = []
    for g0 in range(0, U, group):
        for p in parts:
            a, b = chunks[(p, g0)]
            inter.append(f"{lbl(p, g0)}:")
            inter.extend(lines[a:b])
            inter.append(f"\ts_branch {lbl(p, g0 + group)}" if g0 + group < U else "")
            if g0 + group >= U:  # the last chunk: back to the part's epilogue (far away)
                inter.extend(longbr(lbl(p, U), f"e{p}"))
    out = []
    i = 0
    for a, b, p in regions:
        out.extend(lines[i:a])
        out.extend(longbr(lbl(p, 0), f"s{p}"))  # the prologue jumps to the part's first chunk
        if p == first:
            out.extend(inter)
        out.append(f"{lbl(p, U)}:")
        i = b
    out.extend(lines[i:])
    out = relax(out)
    open(dst, "w").write("\n".join(out))
    print(f"{src}: {len(parts)} parts x {U} units, {len(chunks)} chunks (group {group}) -> {dst}")


BR = re.compile(r"^\s*(s_cbranch_\w+|s_branch)\s+(\.L\w+)\s*$")
LABEL = re.compile(r"^(\.L\w+):")
UNCOND = re.compile(r"^\s*(s_branch|s_setpc_b64|s_endpgm)\b")


def relax(lines):
    """Branches whose target may now be out of s_branch range (+-128 KB): every branch to a label
    more than 16K lines away is rewritten -- s_branch into a long branch in place, s_cbranch_* into
    a short branch to a trampoline (a long branch) placed after the next unconditional transfer,
    where no fall-through reaches it."""
    where = {}
    for i, l in enumerate(lines):
        m = LABEL.match(l)
        if m:
            where[m.group(1)] = i
    tramps = {}  # line index after which to insert -> list of lines
    out_lines = list(lines)
    n = 0
    for i, l in enumerate(lines):
        m = BR.match(l)
        if not m or m.group(2) not in where or abs(where[m.group(2)] - i) < 16000:
            continue
        op, tgt = m.group(1), m.group(2)
        n += 1
        seq = ["\ts_getpc_b64 s[44:45]", f".Lshu_rpc{n}:",
               f"\ts_add_u32 s44, s44, ({tgt}-.Lshu_rpc{n})&4294967295",
               f"\ts_addc_u32 s45, s45, ({tgt}-.Lshu_rpc{n})>>32", "\ts_setpc_b64 s[44:45]"]
        if op == "s_branch":
            out_lines[i] = "\n".join(seq)
            continue
        j = i + 1
        while j < len(lines) and not UNCOND.match(lines[j]):
            j += 1
        assert j < len(lines) and j - i < 16000, "no place for a trampoline"
        out_lines[i] = f"\t{op} .Lshu_tr{n}"
        tramps.setdefault(j, []).extend([f".Lshu_tr{n}:"] + seq)
    res = []
    for i, l in enumerate(out_lines):
        res.append(l)
        if i in tramps:
            res.extend(tramps[i])
    print(f"relaxed {n} branches")
    return "\n".join(res).split("\n")


if __name__ == "__main__":
    main()
