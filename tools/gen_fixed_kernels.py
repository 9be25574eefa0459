#!/usr/bin/env python3
"""Generate compile-time-scheduled bitmatrix kernels: shorthair_amd/csrc/gen/fixed_k<k>_m<m>.hip.

For a fixed (k, m) the generator matrix is a constant (reference cauchy_matrix(),
cauchy_256.cpp:423-481, depends only on k and m), so the whole bitmatrix product (reference
win_encode, cauchy_256.cpp:1398-1477) can be scheduled at build time with every operand a
register name. The reference's 4-bit window method costs 22 table XORs + one 3-input XOR per
output row per input block (86 per 8-row part and block). Round 4 replaces it with straight-line
XOR programs found by a greedy shortest-linear-program search (tools/xor_sched.py) over UNITS of
two consecutive input blocks: a 3-input XOR can then take one word of each block, so most output
rows cost one op per two blocks, plus ~14 shared intermediates per block -- ~62 ops per part and
block at (200, 32) (VALU per launch 3.94e8 -> 3.0e8). Every XOR is emitted as a bitop3 intrinsic
(X3 = truth table 0x96) or a 2-input `^` / v_xor_b32 asm (XV): plain `^` chains spanning all k
steps are reassociated by LLVM into trees that keep every loaded word live (256 VGPRs + AGPR
spills even at k=28).

One generated kernel serves two modes (template flag DEC):
  encode       recovery[g][y] = sum_x M(C[y][x]) data[g][x]             (y < m, row 0 = ones)
  decode A     residual[g][y] = R_y + sum_{x received} M(C[y][x]) d_x   (erased x read as zeros;
               R_y streamed through the same ring as m extra steps after the k input steps)
Rows are split into parts of <= 9 rows (<= 72 accumulator VGPRs); the waves of one workgroup
run the parts of the same columns and read the same LDS ring slots.

Usage: python tools/gen_fixed_kernels.py            (all configs in CONFIGS)
Run by shorthair_amd/build.py before compiling; the generated files are not committed.
"""
import os
import sys

ROOT = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
if os.path.dirname(os.path.abspath(__file__)) not in sys.path:  # tools/xor_sched.py
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
OUTDIR = os.path.join(ROOT, "shorthair_amd", "csrc", "gen")

# (k, m): BASELINE.json configs -- headline (200,32), C2 (64,16), C4 sweep (28,4),(112,16),(224,32)
# -- and the shapes catid/shorthair's own caller issues: Shorthair.cpp:502-504 clamps m to 256-k,
# so its Tester runs k=200/m=56 and k=190/m=66. (216, 40) = (256 - m, m): with the
# k < K dispatch (sh::fixed_kernel_k) it codes every k in [130, 216] of m = 40, the sweep's
# off-grid (150, 40) included (profiles/r06/ab_runs.txt block 14).
CONFIGS = [(200, 32), (64, 16), (28, 4), (112, 16), (224, 32), (200, 56), (190, 66), (216, 40)]
if os.environ.get("SH_CONFIGS"):  # experiments: e.g. SH_CONFIGS="200,32;64,16"
    CONFIGS = [tuple(map(int, c.split(","))) for c in os.environ["SH_CONFIGS"].split(";")]
ROWS_PER_PART = int(os.environ.get("SH_ROWS_PER_PART", "8"))
READ_PIN = os.environ.get("SH_READ_PIN", "0") == "1"
READ_LATE = os.environ.get("SH_READ_LATE", "1") == "1"
# Measurement-only ablations for A/B libraries built by tools/build_variant.sh (never the product
# default, results are wrong), comma-separated: "nodma" = no input DMA (compute on whatever the
# ring holds), "novalu" = DMA, ring reads, barriers and stores but no XOR work, "nobar" = no
# vmcnt wait / barrier (only meaningful with nodma), "nostore" = no output stores, "samecode" =
# every part-wave runs part 0's body (one instruction stream per workgroup instead of P).
ABLATE = set(filter(None, os.environ.get("SH_GEN_ABLATE", "").split(",")))


def gf_tables():
    exp = [0] * 512
    log = [0] * 256
    x = 1
    for i in range(255):
        exp[i] = exp[i + 255] = x
        log[x] = i
        x <<= 1
        if x & 0x100:
            x ^= 0x187
    return exp, log


EXP, LOG = gf_tables()


def gmul(a, b):
    return 0 if a == 0 or b == 0 else EXP[LOG[a] + LOG[b]]


def _tables():
    """Decode the generator-table data the product ships (csrc/cauchy_tables_data.h)."""
    import re
    text = open(os.path.join(ROOT, "shorthair_amd", "csrc", "cauchy_tables_data.h")).read()
    out = {}
    for m in re.finditer(r"static const char SH_TABLE_(\w+)_HEX\[\] =\s*((?:\s*\"[0-9a-f]*\")+);", text):
        out[m.group(1)] = bytes.fromhex("".join(re.findall(r'"([0-9a-f]*)"', m.group(2))))
    return out


def generator(k, m):
    """Full m x k generator (row 0 = ones), restating the reference's cauchy_matrix()
    (cauchy_256.cpp:423-481) exactly as csrc/cauchy_math.hpp does."""
    rows = [[1] * k]
    if m < 2:
        return rows
    t = _tables()
    if m <= 6:
        stat, stride = t[str(m)], 256 - m
        rows += [list(stat[(y - 1) * stride:(y - 1) * stride + k]) for y in range(1, m)]
        return rows
    n = m - 7
    X = t["X"][n * 249 - n * (n + 1) // 2:]
    Y = t["Y"]
    inv = [0] + [EXP[(255 - LOG[a]) % 255] for a in range(1, 256)]

    def div(a, b):
        return 0 if a == 0 or b == 0 else EXP[LOG[a] + 255 - LOG[b]]
    for y in range(1, m):
        G = Y[y - 1]
        rows.append([inv[1 ^ G]] + [div(X[x - 1], X[x - 1] ^ G) for x in range(1, k)])
    return rows


def row_bytes(c):
    out = []
    for _ in range(8):
        out.append(c)
        c = gmul(c, 2)
    return out


class Body:
    """Straight-line code for one part (rows y0..y1-1) over all k inputs."""

    def __init__(self, k, rows, y0, y1, rows_max=None, part=0):
        self.k, self.rows, self.y0, self.y1 = k, rows, y0, y1
        self.part = part
        self.rows_max = rows_max or (y1 - y0)  # the largest part of the kernel (one unit size for all)
        self.lines = []

    def table_expr(self, h, v, have, d):
        """Name of window-table entry v (1..15) of half h, building it if needed (d = name of the
        register set holding this step's 8 input words)."""
        base = {1: f"{d}{4*h+0}", 2: f"{d}{4*h+1}", 4: f"{d}{4*h+2}", 8: f"{d}{4*h+3}"}
        if v in base:
            return base[v]
        name = f"t{h}_{v}"
        if name in have:
            return name
        bits = [b for b in (1, 2, 4, 8) if v & b]
        if len(bits) == 2:  # plain XOR: 4-byte VOP2 encoding (code size is fetch bandwidth)
            self.lines.append(f"    const uint32_t {name} = {base[bits[0]]} ^ {base[bits[1]]};")
        elif len(bits) == 3:
            self.lines.append(f"    const uint32_t {name} = X3({base[bits[0]]}, {base[bits[1]]}, {base[bits[2]]});")
        else:  # 15 = 3 ^ 12
            a = self.table_expr(h, 3, have, d)
            b = self.table_expr(h, 12, have, d)
            self.lines.append(f"    const uint32_t {name} = {a} ^ {b};")
        have.add(name)
        return name

    def unit_code(self, steps, unit, cur):
        """The XOR code of one unit for this part (its rows' accumulators), as lines."""
        save, self.lines = self.lines, []
        L = self.lines
        cols = [t for t in unit if steps[t][0] == "c"]
        L.append("    {")
        if "novalu" in ABLATE:  # keep the loaded words alive, do no XOR work
            L.append("    asm volatile(\"\" :: " + ", ".join(f'"v"({cur}{a})' for a in range(8 * len(cols))) + ");")
        elif cols and JOINT == 0:
            self.window_step(steps[cols[0]][1], cur)
        elif cols:
            self.slp_unit([steps[t][1] for t in cols], cur)
        for j, t in enumerate(unit):
            st = steps[t]
            if st[0] == "r" and self.y0 <= st[1] < self.y1:  # residual row y += the received block R_y
                yi = st[1] - self.y0
                for b in range(8):
                    L.append(f"    XV(acc[{yi}][{b}], {cur}{8 * j + b});")
        # Tie every accumulator to this unit (an empty volatile asm is a chained side effect):
        # otherwise the DAG scheduler floats the pure bitop3 nodes of a ~30K-node basic block
        # away from their loads and keeps every loaded word live.
        for yi in range(self.y1 - self.y0):
            L.append(f"    PIN8(acc[{yi}]);")
        L.append("    }")
        self.lines = save
        return L

    def emit(self, R, S, steps, KP, npf=0, st=0, group=None):
        """group (SH_INTERLEAVE): the Body of every part; the wait / DMA / ring-read code is emitted
        once and each unit's XOR code as an if-chain over the parts, so the part-waves of a
        workgroup walk ONE region of code (each unit's parts adjacent) instead of P separate
        straight-line functions: the instruction fetch of one wave prefetches its neighbours'
        code (round 4: one code stream per workgroup, every part running part 0's code, was 12 %
        faster -- the instruction supply's share)."""
        """Software-pipelined units (see fixed_common.hpp). A unit is JOINT consecutive input
        steps (a pair by default; recovery-row steps are single units) computed as one XOR
        program (tools/xor_sched.py); while unit u computes, the words of unit u+1 are read from
        the ring into the other register bank (dA / dB, 8 words per step). Before reading a unit
        whose steps are not known to have landed, a wave waits (counted vmcnt) for the DMAs of the
        next S steps and joins the workgroup barrier; every wave is then past the units before u,
        so the ring slots of their steps are free and are refilled (up to R steps ahead) right
        there. steps: ("c", x) = input column x (position-table entry x), ("r", y) = decode only:
        the received recovery block of generator row y (entry KP + y), added to row y's residual.
        npf > 0 (persistent encode): a tile after the first finds its steps 0..npf-1 already
        issued by its predecessor, followed by that tile's epilogue stores (st per wave), so
        waits for steps < npf count st more outstanding operations there."""
        L = self.lines
        n = len(steps)
        dma = "nodma" not in ABLATE
        J = unit_steps(R, self.rows_max)

        def tidx(st):
            return st[1] if st[0] == "c" else KP + st[1]

        def uses(st):
            return st[0] == "c" or group is not None or self.y0 <= st[1] < self.y1

        units, i = [], 0
        while i < n:
            if J == 2 and i + 1 < n and steps[i][0] == "c" and steps[i + 1][0] == "c":
                units.append([i, i + 1])
                i += 2
            else:
                units.append([i])
                i += 1
        for bank in ("dA", "dB"):
            L.append("    uint32_t " + ", ".join(f"{bank}{a}" for a in range(8 * J)) + ";")

        def read_unit(u, bank):
            for j, t in enumerate(units[u]):
                if uses(steps[t]):
                    L.append(f"    src.read({t % R}, " + ", ".join(f"{bank}{8 * j + a}" for a in range(8)) + ");")

        nxt_issue = min(n, R - 1)  # steps 0..nxt_issue-1 issued (in order)
        npf = min(npf, nxt_issue)

        def wait(T, I):
            ex = st if T < npf else 0
            return f"    src.template wait<{T}, {I}, {ex}>();" if ex else f"    src.template wait<{T}, {I}>();"

        def consec(a, b):  # steps a..b-1 have consecutive position-table entries
            return all(tidx(steps[a + i]) == tidx(steps[a]) + i for i in range(b - a))
        # Position entries are read 4 steps per LDS read, one burst of issues ahead (Src::pre4);
        # the persistent form (npf > 0) keeps one read per step.
        P4 = npf == 0
        if dma:
            if npf:
                L.append("    if (!src.pref) {")
            for t in range(npf):
                L.append(f"    src.issue({t}, src.pre({tidx(steps[t])}));")
            if npf:
                L.append("    } else {")
                L.append("    src.images_done();")
                L.append("    }")
            if P4:
                chunks = [(c, min(c + 4, nxt_issue)) for c in range(0, nxt_issue, 4)]
                for c0, c1 in chunks:
                    if consec(c0, c1):
                        L.append(f"    const typename Src::Pre4 q{c0} = src.pre4({tidx(steps[c0])});")
                for c0, c1 in chunks:
                    for t in range(c0, c1):
                        L.append(f"    src.issue4({t}, q{c0}, {t - c0});" if consec(c0, c1)
                                 else f"    src.issue({t}, src.pre({tidx(steps[t])}));")
            else:
                for t in range(npf, nxt_issue):
                    L.append(f"    src.issue({t}, src.pre({tidx(steps[t])}));")
        need = units[1][-1] if len(units) > 1 else units[0][-1]
        landed = min(n - 1, max(need, S - 1), nxt_issue - 1)
        assert need <= landed
        L.append(wait(landed, nxt_issue))
        read_unit(0, "dA")
        if nxt_issue < n:
            if P4:
                L.append(f"    typename Src::Pre4 pre4 = src.pre4({tidx(steps[nxt_issue])});")
            else:
                L.append(f"    typename Src::Pre pre = src.pre({tidx(steps[nxt_issue])});")
        b4 = nxt_issue  # first step covered by pre4
        for u, unit in enumerate(units):
            cur, nxt = ("dA", "dB") if u % 2 == 0 else ("dB", "dA")
            L.append("    // ---- " + ", ".join(f"step {t}: " + (f"input block {steps[t][1]}" if steps[t][0] == "c"
                                                                  else f"recovery row {steps[t][1]}") for t in unit))
            if IL_MARK and group is None:  # chunk marker for tools/il_reorder.py (an asm comment)
                L.append(f'    asm volatile(";shu {self.part} {u}");')
            # Pin the unit structure: without this hipcc hoists work across units.
            L.append("    __builtin_amdgcn_sched_barrier(0);")
            if u + 1 < len(units):
                nu = units[u + 1]
                if nu[-1] > landed:
                    # group boundary: the next S steps must have landed (counted vmcnt) and every
                    # wave must be past the units before this one (barrier), which frees their slots
                    landed = min(n - 1, nu[-1] + S - 1, nxt_issue - 1)
                    assert nu[-1] <= landed, "ring too small for the unit size"
                    if "nobar" not in ABLATE:
                        L.append(wait(landed, nxt_issue))
                    issued = False
                    while nxt_issue < n and nxt_issue - R <= unit[0] - 1:
                        if dma and P4:
                            x = nxt_issue
                            if x - b4 < 4 and consec(b4, x + 1):
                                L.append(f"    src.issue4({x}, pre4, {x - b4});")
                            else:
                                L.append(f"    src.issue({x}, src.pre({tidx(steps[x])}));")
                        elif dma:
                            L.append(f"    src.issue({nxt_issue}, pre);")
                        nxt_issue += 1
                        issued = True
                        if nxt_issue < n and not P4:
                            L.append(f"    pre = src.pre({tidx(steps[nxt_issue])});")
                    if P4 and issued and nxt_issue < n:
                        L.append(f"    pre4 = src.pre4({tidx(steps[nxt_issue])});")
                        b4 = nxt_issue
                if not READ_LATE:
                    read_unit(u + 1, nxt)
                if READ_PIN:
                    # keep the next unit's ds_reads at the top of the unit: left free, the
                    # scheduler sinks them to ~25 VALU before their use (LDS latency exposed)
                    L.append("    __builtin_amdgcn_sched_barrier(0);")
            if group is None:
                L.extend(self.unit_code(steps, unit, cur))
            else:
                chain = [(pi, b.unit_code(steps, unit, cur)) for pi, b in enumerate(group)]
                # parts with XOR work in this unit (decode's recovery-row steps touch one part)
                chain = [(pi, c) for pi, c in chain
                         if any(l.strip() not in ("{", "}") and not l.strip().startswith("PIN8") for l in c)]
                for ci, (pi, c) in enumerate(chain):
                    kw = "if" if ci == 0 else "else if"
                    L.append(f"    {kw} (part == {pi})")
                    L.extend(c)
            if READ_LATE and u + 1 < len(units):
                # the next unit's words are read after this unit's XORs (its words are dead
                # then): the two banks are never live together
                L.append("    __builtin_amdgcn_sched_barrier(0);")
                read_unit(u + 1, nxt)
        if IL_MARK and group is None:
            L.append("    __builtin_amdgcn_sched_barrier(0);")
            L.append(f'    asm volatile(";shu {self.part} end");')
        return "\n".join(L)

    def window_step(self, x, cur):
        """One input block with the reference's 4-bit window tables (SH_JOINT=0, A/B only):
        22 table XORs + one bitop3 per output row."""
        L = self.lines
        have = set()
        # Updates ordered by the high-half table entry: each T1 entry is built right before
        # the updates that use it and dies after them (fewer live table registers).
        ups = []
        for yi in range(self.y1 - self.y0):
            v = self.rows[self.y0 + yi][x]
            for b in range(8):
                ups.append((v >> 4, v & 15, yi, b))
                v = gmul(v, 2)
        ups.sort(key=lambda u: (u[0], u[1]))
        for hi, lo, yi, b in ups:
            acc = f"acc[{yi}][{b}]"
            if lo and hi:
                ta = self.table_expr(0, lo, have, cur)
                tb = self.table_expr(1, hi, have, cur)
                L.append(f"    {acc} = X3({acc}, {ta}, {tb});")
            elif lo:
                L.append(f"    XV({acc}, {self.table_expr(0, lo, have, cur)});")
            elif hi:
                L.append(f"    XV({acc}, {self.table_expr(1, hi, have, cur)});")

    def slp_unit(self, xs, cur):
        """The unit's input blocks xs (1 or 2) as one XOR program: word bit 8j + a is input
        sub-block a of block xs[j] (register {cur}{8j + a}); intermediates are defined right
        before their first use, unused ones never."""
        L = self.lines
        nbits = 8 * len(xs)
        tg = []
        for yi in range(self.y1 - self.y0):
            per = [row_bytes(self.rows[self.y0 + yi][x]) for x in xs]
            for b in range(8):
                tg.append(sum(per[j][b] << (8 * j) for j in range(len(xs))))
        inters, reps = sched(tg, nbits)
        order = {w: i for i, (w, _) in enumerate(inters)}
        ops_of = dict(inters)
        names = {}

        def name(w):
            if w & (w - 1) == 0:
                return f"{cur}{w.bit_length() - 1}"
            if w not in names:
                ops = [name(o) for o in ops_of[w]]
                names[w] = f"t{len(names)}"
                expr = f"{ops[0]} ^ {ops[1]}" if len(ops) == 2 else f"X3({ops[0]}, {ops[1]}, {ops[2]})"
                L.append(f"    const uint32_t {names[w]} = {expr};")
            return names[w]

        ups = [(yi, b, reps[t]) for (yi, b), t in zip(((yi, b) for yi in range(self.y1 - self.y0) for b in range(8)), tg) if t]
        ups.sort(key=lambda u: max(order.get(w, -1) for w in u[2]))
        for yi, b, rep in ups:
            acc = f"acc[{yi}][{b}]"
            ws = [name(w) for w in rep]
            for q in range(0, len(ws) - 1, 2):
                L.append(f"    {acc} = X3({acc}, {ws[q]}, {ws[q + 1]});")
            if len(ws) % 2:
                L.append(f"    XV({acc}, {ws[-1]});")


# XOR programs per unit (tools/xor_sched.py), cached on disk by their exact targets: the greedy
# search costs ~0.1 s per 16-bit unit, ~2,600 units over CONFIGS.
JOINT = int(os.environ.get("SH_JOINT", "2"))  # steps per XOR program; 0 = the reference's window tables
_SCHED = {}


def _sched_hash():
    """The cache file is keyed by the scheduler's source: a change to tools/xor_sched.py starts a
    fresh cache instead of reusing programs the old search produced."""
    import hashlib
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "xor_sched.py"), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:12]


_CACHE = os.path.join(ROOT, "shorthair_amd", "csrc", "gen_cache", f"xor_sched_{_sched_hash()}.json")


def unit_steps(R, rows):
    """Steps per XOR program for a ring of R slots and parts of `rows` rows: pairs need the two
    slots of the unit being prefetched plus DMA in flight beyond the waited group (R >= 8; the
    (28,4) ring has 4), and registers: 8 accumulators per row + the pair's 16 words + its ~20
    live intermediates fit 128 VGPRs up to 8 rows ((190,66)'s 9-row parts spill with pairs; a
    scratch spill's vmcnt wait would also drain the DMA ring)."""
    pair_rows = int(os.environ.get("SH_PAIR_ROWS", "8"))  # 16: pairs for 16-row parts (2 waves/SIMD)
    return 2 if JOINT == 2 and R >= 8 and rows <= pair_rows else 1


def _sched_key(tg, nbits):
    return f"{nbits}:" + ",".join(f"{t:x}" for t in tg)


def check_program(tg, nbits, inters, reps):
    """A (cached) XOR program must be exact: every intermediate is the XOR of its 2-3 operands,
    each operand an input word (one bit) or an earlier intermediate, and every target's
    representation XORs to the target. A corrupt cache entry would otherwise become a wrong
    kernel that only the GPU goldens catch."""
    have = {1 << a for a in range(nbits)}
    for w, ops in inters:
        acc = 0
        assert len(ops) in (2, 3), "intermediate arity"
        for o in ops:
            assert o in have, "operand not yet available"
            acc ^= o
        assert acc == w, "intermediate is not the XOR of its operands"
        have.add(w)
    for t in tg:
        if not t:
            continue
        acc = 0
        for w in reps[t]:
            assert w in have, "representation uses an unknown word"
            acc ^= w
        assert acc == t, "representation does not XOR to its target"


def sched(tg, nbits):
    key = _sched_key(tg, nbits)
    if key not in _SCHED:
        import xor_sched
        _SCHED[key] = xor_sched.compute_key(key)[1]
    inters, reps = _SCHED[key]
    inters = [(w, tuple(ops)) for w, ops in inters]
    reps = {int(t): tuple(r) for t, r in reps.items()}
    check_program(tg, nbits, inters, reps)
    return inters, reps


def load_sched_cache():
    import json
    try:
        _SCHED.update(json.load(open(_CACHE)))
    except (OSError, ValueError):
        pass


def save_sched_cache():
    import json
    os.makedirs(os.path.dirname(_CACHE), exist_ok=True)
    with open(_CACHE + ".tmp", "w") as f:
        json.dump(_SCHED, f)
    os.replace(_CACHE + ".tmp", _CACHE)


def prefetch_schedules(cfgs):
    """Compute every unit's XOR program of `cfgs` that the cache lacks, on all host cores."""
    if JOINT == 0:
        return
    keys = set()
    for k, m in cfgs:
        rows = generator(k, m)
        P, _, R = shape(k, m)[:3]
        J = unit_steps(R, -(-m // P))
        base, extra = divmod(m, P)
        y0 = 0
        for p in range(P):
            y1 = y0 + base + (1 if p < extra else 0)
            units = [list(range(x, min(k, x + J))) for x in range(0, k, J)]
            for xs in units:
                tg = []
                for y in range(y0, y1):
                    per = [row_bytes(rows[y][x]) for x in xs]
                    tg += [sum(per[j][b] << (8 * j) for j in range(len(xs))) for b in range(8)]
                keys.add(_sched_key(tg, 8 * len(xs)))
            y0 = y1
    todo = sorted(k for k in keys if k not in _SCHED)
    if todo:
        import multiprocessing as mp
        import xor_sched
        with mp.get_context("fork").Pool(max(1, min(16, os.cpu_count() or 1))) as pool:
            for key, val in pool.imap_unordered(xor_sched.compute_key, todo, chunksize=8):
                _SCHED[key] = val
        save_sched_cache()


def shape(k, m):
    """(P parts, CW column waves, R ring slots, waves/SIMD the registers are allocated for, S).
    <= ROWS_PER_PART rows per part (8 rows = 64 accumulator VGPRs: ~100 VGPRs, 4 waves/SIMD; the
    window tables are rebuilt per part, +22 ops per part and step).
    A workgroup's wave count must be a multiple of the CU's 4 SIMDs: otherwise one SIMD carries an
    extra wave of every workgroup and paces it. So P in {1, 2, 4} with CW = 8 / P (8 waves, two
    workgroups per CU); any other P becomes 8 parts of <= 9 rows with CW = 2 (16 waves, one
    workgroup per CU with a 128 KB ring): (190,66,1336) encode 0.919 vs 1.266 ms and stage A 1.034
    vs 1.335 ms against 9 one-column-wave parts (9 waves, one workgroup per CU); (200,56,1352)
    0.883 vs 0.957 / 0.967 vs 1.000 ms against 7 parts (7 waves)."""
    P = (m + ROWS_PER_PART - 1) // ROWS_PER_PART
    rbytes = int(os.environ.get("SH_RING_BYTES", "65536"))  # > 64 KB: with -DSH_RING_LIMIT (experiments)
    minw_default = None
    if "SH_CW" not in os.environ and P not in (1, 2, 4):
        if m > 72:
            raise ValueError(f"no balanced part layout for m={m} (at most 8 parts of 9 rows)")
        P, CW, rbytes, minw_default = 8, 2, 131072, "4"
    else:
        # Up to 16 waves per workgroup: the CW waves of one part run the SAME straight-line code in
        # lockstep (one barrier per step), so they share every instruction-cache line they fetch.
        # Two parts take CW = 2 and a 48 KB ring (R = 12, three 4-wave workgroups per CU): encode
        # (64,16,1400) 0.122 vs 0.131 ms at 4,096 groups, (112,16,1400) 0.40 vs 0.46 ms, against
        # CW = 4 with two 8-wave workgroups (round-4 A/B, profiles/r04/ab_runs.txt block 7).
        CW = int(os.environ.get("SH_CW", str(2 if P == 2 else max(1, min(8, 8 // P)))))
        if P == 2 and "SH_CW" not in os.environ and "SH_RING_BYTES" not in os.environ:
            rbytes = 49152
    # LDS per workgroup: ring of R slots (the 2 KB per wave of store scratch aliases the ring after
    # the last step)
    slot = 8 * CW * 64 * 4
    if blk_sub(k, m):  # BlkSrc: NG whole block images per slot (fixed_common.hpp BlkGeo)
        sub = blk_sub(k, m)
        nq = (((sub + 3) // 4) + 3) & ~3
        gs = ((8 * sub) + 15) & ~15
        while (gs // 4) % 32 != nq % 32:
            gs += 16
        ng = (127 + nq - 1) // nq + 1
        slot = -(-ng * gs // 1024) * 1024
    rmax = int(os.environ.get("SH_RING_MAX", "19" if rbytes <= 65536 else "16"))
    R = int(os.environ.get("SH_RING", str(max(3, min(rmax, rbytes // slot, max(76 * 1024, rbytes) // slot)))))
    rows = (m + P - 1) // P
    minw = int(os.environ.get("SH_MIN_WAVES", minw_default or ("2" if rows > 12 else ("3" if rows > 8 else "4"))))
    # blocks per barrier: R >= 2*SYNC + 1 keeps >= 1 group of DMA in flight past the one waited for
    sync = int(os.environ.get("SH_SYNC", str(max(1, min(4, (R - 1) // 2 - 1)))))
    if stream_mode(P):
        R = int(os.environ.get("SH_STREAM_R", "6"))  # register buffers: steps loaded ahead
    return P, CW, R, minw, sync


def parts_per_wg(P):
    """Parts per workgroup (fixed_common.hpp Shape::PW). A/B switch SH_PW: the P parts of a tile
    run in P / SH_PW workgroups, each with its own ring over the whole tile (one or two code
    streams per workgroup for P / PW times the input reads through L2). Default: all P."""
    pw = int(os.environ.get("SH_PW", "0")) or P
    return pw if P % pw == 0 else P


def blk_sub(k, m):
    """Whole-block input ring (fixed_common.hpp BlkSrc) for B = 8 * SH_BLK, A/B switch: the
    kernel then serves that block size only. 0 = the sub-block-row gather (Src)."""
    return int(os.environ.get("SH_BLK", "0"))


def split_tiles(mode, k, P, pers):
    """Split-tile programs (fixed_common.hpp RowSink "Split tiles": the launch's last tiles run
    as two half-step workgroups combined in-launch), A/B switch SH_SPLIT_GEN=1: bit-exact but no
    faster (profiles/r06/ab_runs.txt block 2), and the half programs triple the generated code
    and the build time, so the product generates none."""
    if os.environ.get("SH_SPLIT_GEN", "0") != "1" or pers or RINIT or INTERLEAVE or stream_mode(P):
        return False
    return k >= 16


# A/B switch SH_ROW_PAIRS=1: two rows per epilogue barrier (RowSink::row2)
ROW_PAIRS = os.environ.get("SH_ROW_PAIRS", "0") == "1"
# A/B switch SH_L2PF=N: encode epilogues touch the first N steps of a later tile (Src::l2_prefetch)
L2PF = int(os.environ.get("SH_L2PF", "0"))

PERSIST = os.environ.get("SH_PERSIST", "0") == "1"
# Decode stage A, SH_RINIT=1 (measured, not the default): residual rows start as the recovery
# blocks R_y, loaded into the accumulators in the prologue (Src::rrow) instead of m extra ring
# steps -- same time (ab_runs.txt block 7), but the per-lane dword loads fetch those rows at
# ~1.6x their bytes (stage A reads 2.63 vs 2.42 GB per launch).
RINIT = os.environ.get("SH_RINIT", "0") == "1"


PERSIST_DEC = os.environ.get("SH_PERSIST_DEC", "1") == "1"


def persistent(mode, P, R):
    """Persistent workgroups with next-tile prefetch (fixed_common.hpp SH_PERSISTENT_TILES) for
    kernels whose ring keeps >= 4 slots below the 2P row images; decode stage A stages the next
    tile's position tables into LDS at the end of each tile."""
    return (PERSIST and (mode == "enc" or PERSIST_DEC) and not stream_mode(P) and R - 2 * P >= 4
            and "nodma" not in ABLATE)


def stream_mode(P):
    """One-part shapes may load each lane's words straight into registers (StreamSrc in
    fixed_common.hpp) instead of through the LDS ring."""
    mode = os.environ.get("SH_STREAM", "0")
    return mode == "all" or (P == 1 and mode == "1")


def gen_config(k, m):
    rows = generator(k, m)
    P, CW, R, minw, sync = shape(k, m)
    # balanced parts: sizes differ by at most one row (the slowest part paces the barriers)
    base, extra = divmod(m, P)
    parts, y0 = [], 0
    for p in range(P):
        n = base + (1 if p < extra else 0)
        parts.append((y0, y0 + n))
        y0 += n
    name = f"k{k}_m{m}"
    out = [f"// GENERATED by tools/gen_fixed_kernels.py -- do not edit. (k={k}, m={m})",
           "// Compile-time-scheduled windowed bitmatrix product for one generator; see the",
           "// generator's docstring and DESIGN.md.",
           "#pragma once",
           '#include "../fixed_common.hpp"',
           "",
           "namespace sh {",
           "namespace fixed {",
           ""]
    KP = (k + 3) & ~3
    pers = {mode: persistent(mode, P, R) for mode in ("enc", "dec")}
    split = {mode: split_tiles(mode, k, P, pers[mode]) for mode in ("enc", "dec")}
    for mode in ("enc", "dec"):
        rinit = mode == "dec" and RINIT and not pers[mode]
        steps = [("c", x) for x in range(k)] + ([("r", y) for y in range(m)] if mode == "dec" and not rinit else [])
        if INTERLEAVE and not pers[mode] and not rinit and len(parts) > 1:
            out.extend(interleaved_function(name, mode, k, rows, parts, R, sync, steps, KP))
            out.extend(["template <class Src, class Snk>",
                        f"__device__ __forceinline__ void run_{name}_{mode}_half(int half, int part, const Src &src, const Snk &sink) {{",
                        f"    run_{name}_{mode}(part, src, sink);", "}", ""])
            continue
        nrmax = max(b - a for a, b in parts)

        def body_fn(fname, p, y0, y1, sub_steps, split_half=None, step0=0):
            """One part's straight-line function over sub_steps; split_half: the epilogue stores a
            partial and the second arriving half combines (RowSink "Split tiles")."""
            # epilogue stores per wave: two 16-byte pieces per row of its part (RowSink::row)
            npf = R - 2 * P if pers[mode] else 0
            body = Body(k, rows, y0, y1, nrmax, part=p).emit(R, sync, sub_steps, KP, npf=npf,
                                                             st=2 * (y1 - y0))
            nr = y1 - y0
            out.append(f"template <class Src, class Snk>")
            out.append(f"__device__ __forceinline__ void {fname}(const Src &src, const Snk &sink) {{")
            out.append(f"    uint32_t acc[{nr}][8];")
            if step0:
                out.append(f"    src.set_step0({step0});  // encode: this half's first input block")
            # opaque zeros: a constant 0 would be folded into the first step, whose pinned results
            # then need register copies of shared table entries (AGPR spills at k=200).
            if rinit:
                out.extend(f"    src.rrow({y0 + yi}, acc[{yi}]);" for yi in range(nr))
            else:
                out.append(f"    for (int y = 0; y < {nr}; ++y) for (int b = 0; b < 8; ++b) ZERO(acc[y][b]);")
            out.append(body)
            out.append("    __builtin_amdgcn_sched_barrier(0);")
            out.append(f"    // epilogue: store rows {y0}..{y1 - 1}" + (" (partial of a split tile)" if split_half is not None else ""))
            out.append("    src.release();  // the store scratch aliases the ring")
            if L2PF and mode == "enc" and not pers[mode] and split_half is None:
                out.append(f"    const auto l2pf = src.template l2_prefetch<{L2PF}>();  // A/B: warm L2 for a later tile")
            if pers[mode]:
                out.append(f"    src.prefetch_next({R - 2 * P});  // the next tile's first steps")
            out.append("    sink.prepare();")
            # row pairs (A/B switch): not with the persistent form (its images sit in the ring's
            # top 2P slots) nor the split tiles' partial rows
            pairs = ROW_PAIRS and not pers[mode] and split_half is None and 4 * parts_per_wg(P) <= R
            for yi in range(nrmax):  # every part joins the same number of row barriers
                out.append("    __builtin_amdgcn_sched_barrier(0);")
                last = "true" if yi == nrmax - 1 else "false"
                if yi >= nr and pairs:
                    out.append(f"    sink.template pad2<{yi}, {last}>();")
                elif yi >= nr:
                    out.append(f"    sink.template pad<{yi}>();")
                elif "halfstore" in ABLATE and p >= len(parts) // 2:
                    out.append(f"    asm volatile(\"\" :: " + ", ".join(f'"v"(acc[{yi}][{b}])' for b in range(8)) + ");")
                elif "nostore" in ABLATE:
                    out.append(f"    asm volatile(\"\" :: " + ", ".join(f'"v"(acc[{yi}][{b}])' for b in range(8)) + ");")
                elif split_half is not None:
                    out.append(f"    sink.template part_row<{yi}>({y0 + yi}, acc[{yi}]);")
                elif pairs:
                    out.append(f"    sink.template row2<{yi}, {last}>({y0 + yi}, acc[{yi}]);")
                else:
                    out.append(f"    sink.template row<{yi}>({y0 + yi}, acc[{yi}]);")
            if split_half is not None:
                out.append(f"    sink.combine({y0}, {nr});")
            if L2PF and mode == "enc" and not pers[mode] and split_half is None:
                out.append("    src.l2_done(l2pf);  // the compiler's counted wait: the prefetch loads only")
            out.append("}")
            out.append("")

        for p, (y0, y1) in enumerate(parts):
            body_fn(f"run_{name}_{mode}_p{p}", p, y0, y1, steps)
        # Split tiles: two half-step programs per part (the steps cut at an even index, so the
        # pair units and their XOR programs are those of the whole program)
        n0 = (len(steps) // 2) & ~1
        if split[mode]:
            for h, (sub, x0) in enumerate(((steps[:n0], 0), (steps[n0:], n0 if mode == "enc" else 0))):
                for p, (y0, y1) in enumerate(parts):
                    body_fn(f"run_{name}_{mode}_h{h}_p{p}", p, y0, y1, sub, split_half=h, step0=x0)
        out.append(f"template <class Src, class Snk>")
        out.append(f"__device__ __forceinline__ void run_{name}_{mode}_half(int half, int part, const Src &src, const Snk &sink) {{")
        if split[mode]:
            for h in (0, 1):
                out.append(f"    {'if' if h == 0 else 'else if'} (half == {h}) {{")
                for p in range(len(parts)):
                    kw = "if" if p == 0 else "else if"
                    out.append(f"        {kw} (part == {p}) run_{name}_{mode}_h{h}_p{p}(src, sink);")
                out.append("    }")
        else:  # never launched with split tiles (FIXED_KERNEL SPLIT = 0)
            out.append(f"    run_{name}_{mode}(part, src, sink);")
        out.append("}")
        out.append("")
        out.append(f"template <class Src, class Snk>")
        out.append(f"__device__ __forceinline__ void run_{name}_{mode}(int part, const Src &src, const Snk &sink) {{")
        if "samecode" in ABLATE:  # timing only: every part-wave runs part 0's code (one code stream)
            out.append(f"    run_{name}_{mode}_p0(src, sink);")
        for p in range(len(parts)):
            if "samecode" in ABLATE:
                break
            kw = "if" if p == 0 else "else if"
            out.append(f"    {kw} (part == {p}) run_{name}_{mode}_p{p}(src, sink);")
        out.append("}")
        out.append("")
    out.append("}  // namespace fixed")
    out.append("}  // namespace sh")
    os.makedirs(OUTDIR, exist_ok=True)
    inc = os.path.join(OUTDIR, f"fixed_{name}.inc")
    with open(inc, "w") as f:
        f.write("\n".join(out) + "\n")
    # One translation unit per kernel (encode / decode stage A): each is a ~30K-instruction
    # straight-line function, so the build compiles them in parallel.
    paths = []
    for mode, dec in (("enc", "false"), ("dec", "true")):
        path = os.path.join(OUTDIR, f"fixed_{name}_{mode}.hip")
        with open(path, "w") as f:
            f.write(f"// GENERATED by tools/gen_fixed_kernels.py -- do not edit. (k={k}, m={m}, {mode})\n"
                    f'#include "fixed_{name}.inc"\n'
                    + (f"FIXED_KERNEL_PERSISTENT({name}, {k}, {m}, {P}, {CW}, {R}, {minw}, {mode}, {dec})\n" if pers[mode] else
                       f"FIXED_KERNEL({name}, {k}, {m}, {P}, {CW}, {R}, {minw}, {mode}, {dec}, "
                       f"{'false' if 'nodma' in ABLATE else 'true'}, {'true' if stream_mode(P) else 'false'}, "
                       f"{parts_per_wg(P)}, {blk_sub(k, m)}, {1 if split[mode] else 0})\n"))
        paths.append(path)
    return paths


INTERLEAVE = os.environ.get("SH_INTERLEAVE", "0") == "1"
# Unit markers (asm comments ";shu <part> <unit>") for the code-layout pass tools/il_reorder.py
IL_MARK = os.environ.get("SH_IL_MARK", "0") == "1"


def interleaved_function(name, mode, k, rows, parts, R, sync, steps, KP):
    """run_<name>_<mode>(part, src, sink) as ONE function: the ring code once, each unit's XOR
    code an if-chain over the parts (Body.emit group=...), the epilogue's rows by part."""
    nrmax = max(b - a for a, b in parts)
    bodies = [Body(k, rows, y0, y1, nrmax) for y0, y1 in parts]
    body = bodies[0].emit(R, sync, steps, KP, group=bodies)
    base, extra = divmod(sum(b - a for a, b in parts), len(parts))
    out = ["template <class Src, class Snk>",
           f"__device__ __forceinline__ void run_{name}_{mode}(int part, const Src &src, const Snk &sink) {{",
           f"    uint32_t acc[{nrmax}][8];",
           f"    for (int y = 0; y < {nrmax}; ++y) for (int b = 0; b < 8; ++b) ZERO(acc[y][b]);",
           body,
           "    __builtin_amdgcn_sched_barrier(0);",
           "    // epilogue: this part's rows (part p owns rows y0(p) .. y0(p) + nr(p) - 1)",
           "    src.release();  // the store scratch aliases the ring",
           "    sink.prepare();",
           f"    const int y0 = part * {base} + (part < {extra} ? part : {extra});",
           f"    const int nr = {base} + (part < {extra} ? 1 : 0);"]
    for yi in range(nrmax):  # every part joins the same number of row barriers
        out.append("    __builtin_amdgcn_sched_barrier(0);")
        if "nostore" in ABLATE:
            out.append(f"    asm volatile(\"\" :: " + ", ".join(f'"v"(acc[{yi}][{b}])' for b in range(8)) + ");")
        elif all(b - a > yi for a, b in parts):
            out.append(f"    sink.template row<{yi}>(y0 + {yi}, acc[{yi}]);")
        else:
            out.append(f"    if ({yi} < nr) sink.template row<{yi}>(y0 + {yi}, acc[{yi}]);")
            out.append(f"    else sink.template pad<{yi}>();")
    out.append("}")
    out.append("")
    return out


# Snippet table for runtime coefficients (decode stage B, csrc/stageb.hip): snippet c computes
# tmp[b] = T0[lo(c*2^b)] ^ T1[hi(c*2^b)], b = 0..7, from window tables pinned in VGPRs, and
# returns with s_setpc_b64. 256 snippets x 64 B = 16 KB, emitted inside the kernel behind an
# s_branch (file-scope asm is dropped by HIP device compilation).
SNIP_T0, SNIP_T1, SNIP_TMP = 100, 116, 132
# pinned low (v[32:127]) so a stage-B kernel fits 128 VGPRs (4 waves per SIMD)
SNIPA_ACC, SNIPA_T0, SNIPA_T1 = 32, 96, 112


# measurement table for 4-output waves (tools/snip_bench.hip): tables right above the accumulators
SNIPB_REGS = (32, 64, 80)


def acc_table(name, A, T0, T1, chain=False):
    """chain: the snippet advances the VGPR index to the next accumulator set (m0 += 8), shifts the
    queue of snippet addresses s[44:61] down one pair and jumps to the next one (one redirect per
    product; the caller puts 8 addresses + its return address in s[44:61])."""
    low = name.lower()
    stride = 104 if chain else 72
    t = [f"#define SH_{name}_ACC {A}", f"#define SH_{name}_T0 {T0}", f"#define SH_{name}_T1 {T1}",
         f"#define SH_{name}_STRIDE {stride}", f"#define SH_{name}_NULL 256",
         f'#define SH_{name}_TABLE(SFX) asm volatile("s_branch sh_{low}_end" #SFX "\\n"',
         '    ".p2align 6\\n"',
         f'    "sh_{low}_base" #SFX ":\\n"']
    for c in range(256):
        v = c
        for b in range(8):
            lo, hi = v & 15, v >> 4
            t.append(f'    "v_bitop3_b32 v{A + b}, v{A + b}, v{T0 + lo}, v{T1 + hi} bitop3:0x96\\n"')
            v = gmul(v, 2)
        if chain:
            t.append('    "s_add_u32 m0, m0, 8\\n"')
            for q in range(8):
                t.append(f'    "s_mov_b64 s[{44 + 2 * q}:{45 + 2 * q}], s[{46 + 2 * q}:{47 + 2 * q}]\\n"')
            t.append('    "s_setpc_b64 s[44:45]\\n"')
        else:
            t.append('    "s_setpc_b64 s[40:41]\\n"')
            t.append('    "s_nop 0\\n"')
    if chain:  # null entry: same queue step, no XOR work
        t.append('    "s_add_u32 m0, m0, 8\\n"')
        for q in range(8):
            t.append(f'    "s_mov_b64 s[{44 + 2 * q}:{45 + 2 * q}], s[{46 + 2 * q}:{47 + 2 * q}]\\n"')
        t.append('    "s_setpc_b64 s[44:45]\\n"')
    else:
        t.append('    "s_setpc_b64 s[40:41]\\n"')
    t.append(f'    "sh_{low}_end" #SFX ":\\n" ::: "memory")')
    return t


def gen_snippets():
    lines = ["// GENERATED by tools/gen_fixed_kernels.py -- do not edit.",
             "// 256 compile-time 'multiply by c' snippets (see csrc/stageb.hip).",
             "#pragma once",
             f"#define SH_SNIP_T0 {SNIP_T0}",
             f"#define SH_SNIP_T1 {SNIP_T1}",
             f"#define SH_SNIP_TMP {SNIP_TMP}",
             '#define SH_SNIPPET_TABLE(SFX) asm volatile("s_branch sh_snip_end" #SFX "\\n"',
             '    ".p2align 6\\n"',
             '    "sh_snip_base" #SFX ":\\n"']
    for c in range(256):
        v = c
        lines.append('    ".p2align 6\\n"')
        for b in range(8):
            lo, hi = v & 15, v >> 4
            lines.append(f'    "v_xor_b32 v{SNIP_TMP + b}, v{SNIP_T0 + lo}, v{SNIP_T1 + hi}\\n"')
            v = gmul(v, 2)
        lines.append('    "s_setpc_b64 s[40:41]\\n"')
    lines.append('    "sh_snip_end" #SFX ":\\n" ::: "memory")')
    # Accumulating variant for VGPR-index mode (csrc/stageb.hip, stageb_fixed): snippet c does
    # acc[b] ^= T0[lo(c*2^b)] ^ T1[hi(c*2^b)] as 8 v_bitop3_b32 whose destination and first
    # source are relative to M0 (s_set_gpr_idx_on ..., gpr_idx(SRC0,DST)): the caller selects the
    # output row with s_set_gpr_idx_idx, no copy-and-XOR of a temporary. Every snippet is exactly
    # SNIPA_STRIDE = 72 bytes (8 x 8-byte bitop3 + s_setpc + s_nop), so snippet c sits at
    # base + 72*c; entry 256 is the null snippet (zero coefficient / unused output: return at once).
    # The decode setup writes absolute snippet addresses, so the stage-B loop computes no targets.
    acc = acc_table("SNIPA", SNIPA_ACC, SNIPA_T0, SNIPA_T1)
    accb = acc_table("SNIPB", *SNIPB_REGS)
    accc = acc_table("SNIPC", SNIPA_ACC, SNIPA_T0, SNIPA_T1, chain=True)
    with open(os.path.join(OUTDIR, "snippets.h"), "w") as f:
        f.write(lines[0] + "\n" + lines[1] + "\n" + lines[2] + "\n" + "\n".join(lines[3:6]) + "\n"
                + " \\\n".join(lines[6:]) + "\n")
        for t in (acc, accb, accc):
            f.write("\n".join(t[:5]) + "\n" + " \\\n".join(t[5:]) + "\n")


# Column snippets for the runtime-coefficient tile kernels at m >= 7 (csrc/tile_snip.hip). There
# the generator is C[y][x] = X'_x / (X'_x + Y'_y) with Y'_y = Y[y-1] the SAME for every m (only X'
# depends on m, cauchy_256.cpp:453-477), so the coefficients of 4 consecutive rows for input x
# are a function of one byte, v = X'_x. Snippet (block r, v) applies M(C[y][x]) for the rows
# y = 4r..4r+3 to accumulator sets 4*(r%2)..+3 (v[32+32*(r%2)+8j+b]) from the window tables in
# v[96:127] (v96 = v112 = 0): 32 v_bitop3_b32 and a return, no VGPR-index mode -- one call per 4
# rows and input instead of one per row (the index mode alone costs 1.8x).
# 64 blocks (rows 0..255) x 256 values, COL_STRIDE bytes each, in COL_TUS translation units of
# COL_BLOCKS_PER_TU blocks; TU 0 also holds 8 "unit" snippets (acc set s ^= the input: decode
# stage A's recovery-row steps) and a null snippet, at block COL_BLOCKS_PER_TU.
COL_STRIDE, COL_TUS, COL_BLOCKS_PER_TU = 264, 4, 16


def _col_snippet(lines, accs, coefs, label=None):
    for j, c in enumerate(coefs):
        v = c
        for b in range(8):
            if c:
                lo, hi = v & 15, v >> 4
                lines.append(f"v_bitop3_b32 v{accs[j] + b}, v{accs[j] + b}, v{SNIPA_T0 + lo}, v{SNIPA_T1 + hi} bitop3:0x96")
            v = gmul(v, 2)
    n = sum(8 for c in coefs if c)
    lines.append("s_setpc_b64 s[40:41]")
    lines.append(f".skip {COL_STRIDE - 8 * n - 4}")  # fixed stride (never executed): base + COL_STRIDE * index


_COL_Y = None


def col_coef(y, v):
    """Generator coefficient of row y (m >= 7) for an input whose Cauchy parameter X'_x is v:
    row 0 = ones, else X'/(X' + Y[y-1]) (cauchy_256.cpp:453-477; 0 where the reference's divide
    would see a zero operand)."""
    global _COL_Y
    if _COL_Y is None:
        _COL_Y = list(_tables()["Y"]) + [0] * 256
    if y == 0:
        return 1
    b = v ^ _COL_Y[y - 1]
    return 0 if v == 0 or b == 0 else EXP[LOG[v] + 255 - LOG[b]]


def cauchy_xp(k, m):
    """X'_x of the m >= 7 generator (X'_0 = 1, X'_x = X[x-1] at offset n*249 - n(n+1)/2, n = m-7)."""
    n = m - 7
    X = _tables()["X"][n * 249 - n * (n + 1) // 2:]
    return [1] + [X[x - 1] for x in range(1, k)]


def gen_colsnips():
    coef = col_coef
    for tu in range(COL_TUS):
        L = []
        for rl in range(COL_BLOCKS_PER_TU):
            r = tu * COL_BLOCKS_PER_TU + rl
            accs = [SNIPA_ACC + 32 * (r % 2) + 8 * j for j in range(4)]
            for v in range(256):
                L.append(".p2align 3")
                _col_snippet(L, accs, [coef(4 * r + j, v) for j in range(4)])
        if tu == 0:
            for st in range(8):  # unit snippets: acc set st ^= the input block (coefficient 1)
                L.append(".p2align 3")
                _col_snippet(L, [SNIPA_ACC + 8 * st], [1])
            L.append(".p2align 3")
            _col_snippet(L, [], [])  # null snippet
        body = "\n".join(f'    "{l}\\n"' for l in L)
        src = f"""// GENERATED by tools/gen_fixed_kernels.py -- do not edit. Column snippets, blocks
// {tu * COL_BLOCKS_PER_TU}..{tu * COL_BLOCKS_PER_TU + COL_BLOCKS_PER_TU - 1} (rows {4 * tu * COL_BLOCKS_PER_TU}..{4 * (tu + 1) * COL_BLOCKS_PER_TU - 1}); see the generator.
#include <hip/hip_runtime.h>
#include <stdint.h>
namespace sh {{
// Holds the table; its only launch reports where the table was loaded.
__global__ void colsnip_probe_{tu}(uint64_t *out) {{
    // the table is ~1 MB: jump over it with an absolute (computed) jump, s_branch reaches 128 KB
    asm volatile("s_getpc_b64 s[42:43]\\n"
    "s_add_u32 s42, s42, sh_colsnip_end{tu}@rel32@lo+4\\n"
    "s_addc_u32 s43, s43, sh_colsnip_end{tu}@rel32@hi+12\\n"
    "s_setpc_b64 s[42:43]\\n"
    ".p2align 6\\n"
    "sh_colsnip_base{tu}:\\n"
{body}
    "sh_colsnip_end{tu}:\\n" ::: "s42", "s43", "scc", "memory");
    uint64_t base;
    asm volatile(
        "s_getpc_b64 s[42:43]\\n"
        "s_add_u32 s42, s42, sh_colsnip_base{tu}@rel32@lo+4\\n"
        "s_addc_u32 s43, s43, sh_colsnip_base{tu}@rel32@hi+12\\n"
        "s_mov_b64 %0, s[42:43]"
        : "=s"(base)
        :
        : "s42", "s43", "scc");
    if (threadIdx.x == 0) *out = base;
}}
}}  // namespace sh
"""
        with open(os.path.join(OUTDIR, f"colsnip_{tu}.hip"), "w") as f:
            f.write(src)
    with open(os.path.join(OUTDIR, "colsnip.h"), "w") as f:
        f.write("// GENERATED by tools/gen_fixed_kernels.py -- column-snippet table layout.\n#pragma once\n"
                f"#define SH_COL_STRIDE {COL_STRIDE}\n#define SH_COL_TUS {COL_TUS}\n"
                f"#define SH_COL_BLOCKS_PER_TU {COL_BLOCKS_PER_TU}\n"
                "#define SH_COL_UNIT(s) ((SH_COL_BLOCKS_PER_TU * 256 + (s)) * SH_COL_STRIDE)  /* offset in TU 0 */\n"
                "#define SH_COL_NULL ((SH_COL_BLOCKS_PER_TU * 256 + 8) * SH_COL_STRIDE)\n")


def main(argv=()):
    cfgs = CONFIGS
    if argv:
        cfgs = [tuple(map(int, a.split(","))) for a in argv]
    load_sched_cache()
    prefetch_schedules(cfgs)
    paths = [p for (k, m) in cfgs for p in gen_config(k, m)]
    gen_snippets()
    gen_colsnips()
    # registry of generated shapes
    reg = ["// GENERATED by tools/gen_fixed_kernels.py -- list of compile-time-scheduled (k, m).",
           "#pragma once", "#define SH_FIXED_CONFIGS(X) \\"]
    reg += [f"    X({k}, {m}) \\" for (k, m) in CONFIGS]
    reg.append("")
    with open(os.path.join(OUTDIR, "fixed_configs.h"), "w") as f:
        f.write("\n".join(reg) + "\n")
    for p in paths:
        print("wrote", os.path.relpath(p, ROOT))


if __name__ == "__main__":
    main(sys.argv[1:])
