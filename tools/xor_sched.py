#!/usr/bin/env python3
"""XOR programs for one compile-time step of the bitsliced bitmatrix product.

A step of a part-wave applies one input block x to the part's rows: for every output sub-block
row (y, b) the lane does acc[y][b] ^= XOR of the input words d_a whose bit a is set in the
8-bit mask t = C[y][x] * 2^b (GF(256)/0x187; the reference's 8x8 submatrix semantics,
cauchy_256.cpp:1398-1477 / :1553-1568). The reference's 4-bit window method (win_encode) builds
both 4-input window tables (22 XORs) and spends one 3-input XOR per row: 22 + rows*8 ops.

Here the step is scheduled as a small shortest-linear-program instead: a set S of intermediate
words (each ONE v_bitop3_b32 / v_xor_b32 of 2 or 3 earlier words) is chosen so that every
target is a XOR of as few words of S + inputs as possible; a target of n words costs ceil(n/2)
accumulating ops (acc ^ a ^ b per op). Greedy: repeatedly add the candidate (XOR of 2 or 3
available words) that lowers the step's total op count most. With D[v] = the fewest available
words summing to v, adding word c gives D'[v] = min(D[v], 1 + D[v ^ c]) exactly (a minimal sum
uses c at most once), so every candidate is priced with one vectorised lookup.

Measured on the (200, 32) generator: 86 -> ~77 ops per part-step (8 rows) on average.
"""
import itertools

import numpy as np

_BIG = 99


def _dist_of(elems):
    """D[v] = fewest elements of `elems` XOR-ing to v, and one such representation per v."""
    D = np.full(256, _BIG, np.int32)
    D[0] = 0
    rep = {0: ()}
    frontier = [0]
    while frontier:
        nxt = []
        for v in frontier:
            for e in elems:
                w = v ^ e
                if D[w] == _BIG:
                    D[w] = D[v] + 1
                    rep[w] = rep[v] + (e,)
                    nxt.append(w)
        frontier = nxt
    return D, rep


def schedule(targets, trials=1, seed=0):
    """targets: list of 8-bit masks (0 = nothing to do). Returns (inters, reps, ops):
    inters = [(mask, (operand masks...))] in creation order (each operand an input 1<<a or an
    earlier intermediate), reps = {target mask: tuple of words}, ops = total op count."""
    T = np.array([t for t in targets if t], np.int64)
    if T.size == 0:
        return [], {}, 0
    best = None
    rng = np.random.default_rng(seed)
    for trial in range(trials):
        avail = [1 << a for a in range(8)]
        D, rep = _dist_of(avail)
        inters = []
        cur = int(((D[T] + 1) // 2).sum())
        while True:
            cands = {}
            for a, b in itertools.combinations(avail, 2):
                cands.setdefault(a ^ b, (a, b))
            for a, b, c in itertools.combinations(avail, 3):
                cands.setdefault(a ^ b ^ c, (a, b, c))
            for a in avail:
                cands.pop(a, None)
            cands.pop(0, None)
            if not cands:
                break
            C = np.fromiter(cands.keys(), np.int64)
            newD = np.minimum(D[T][None, :], 1 + D[T[None, :] ^ C[:, None]])
            cost = ((newD + 1) // 2).sum(axis=1) + 1  # the new word's own op
            lo = cost.min()
            if lo >= cur:
                break
            pick = np.flatnonzero(cost == lo)
            c = int(C[pick[0] if trial == 0 else rng.choice(pick)])
            inters.append((c, cands[c]))
            avail.append(c)
            # exact incremental update of D / rep with the new word
            for v in range(256):
                w = v ^ c
                if D[w] + 1 < D[v]:
                    D[v] = D[w] + 1
                    rep[v] = rep[w] + (c,)
            cur = int(((D[T] + 1) // 2).sum())
        total = cur + len(inters)
        if best is None or total < best[2]:
            best = (inters, {int(t): rep[int(t)] for t in set(T.tolist())}, total)
    return best


_TRI = {}


def _tri(n):
    """Index arrays of all pairs and triples of n items (cached)."""
    if n not in _TRI:
        p = np.array(list(itertools.combinations(range(n), 2)), np.int64).reshape(-1, 2)
        t = np.array(list(itertools.combinations(range(n), 3)), np.int64).reshape(-1, 3)
        _TRI[n] = (p, t)
    return _TRI[n]


def schedule_joint(targets, nbits, trials=6, seed=0):
    """schedule() over nbits-bit targets (the 8-bit masks of `nbits // 8` consecutive steps
    packed, step j in bits 8j..8j+7): one accumulating op can then take a word of each step
    (acc ^ a_x ^ b_x+1), which the per-step form cannot. D is a dense 2^nbits table (nbits <=
    16). The first trial breaks ties by the lowest candidate, the others at random (seeded:
    the result is deterministic); the cheapest program wins (6 trials: ~4 % fewer ops than one).
    Same return value as schedule()."""
    T = np.array([t for t in targets if t], np.int64)
    if T.size == 0:
        return [], {}, 0
    N = 1 << nbits
    idx = np.arange(N, dtype=np.int64)
    D0 = np.array([bin(v).count("1") for v in range(N)], np.int32)  # sums of the inputs alone
    rng = np.random.default_rng(seed)
    best = None
    for trial in range(trials):
        avail = [1 << a for a in range(nbits)]
        D = D0.copy()
        inters = []
        cur = int(((D[T] + 1) // 2).sum())
        while True:
            A = np.array(avail, np.int64)
            pi, ti = _tri(len(A))
            c2 = A[pi[:, 0]] ^ A[pi[:, 1]]
            c3 = A[ti[:, 0]] ^ A[ti[:, 1]] ^ A[ti[:, 2]]
            C = np.unique(np.concatenate([c2, c3]))
            C = C[D[C] > 1]
            if C.size == 0:
                break
            newD = np.minimum(D[T][None, :], 1 + D[T[None, :] ^ C[:, None]])
            cost = ((newD + 1) // 2).sum(axis=1) + 1  # the new word's own op
            lo = int(cost.min())
            if lo >= cur:
                break
            ties = np.flatnonzero(cost == lo)
            c = int(C[ties[0] if trial == 0 else rng.choice(ties)])
            hit = np.flatnonzero(c2 == c)
            ops = tuple(int(v) for v in A[pi[hit[0]]]) if hit.size else \
                tuple(int(v) for v in A[ti[np.flatnonzero(c3 == c)[0]]])
            inters.append((c, ops))
            avail.append(c)
            D = np.minimum(D, 1 + D[idx ^ c])
            cur = int(((D[T] + 1) // 2).sum())
        if best is None or cur + len(inters) < best[2]:
            best = (inters, avail, cur + len(inters), D)
    inters, avail, total, D = best
    # representations: peel words greedily along D (each step removes one word, D drops by one)
    reps = {}
    for t in set(T.tolist()):
        v, rep = int(t), []
        while v:
            w = next(w for w in avail if D[v ^ w] == D[v] - 1)
            rep.append(w)
            v ^= w
        reps[int(t)] = tuple(rep)
    return inters, reps, total


def compute_key(key):
    """Cache entry of tools/gen_fixed_kernels.py: key "nbits:hex,hex,..." -> (key, JSON-able
    (intermediates, representations)). A module-level function so a process pool can run it."""
    nbits, body = key.split(":")
    tg = [int(t, 16) for t in body.split(",")]
    seed = int.from_bytes(__import__("hashlib").sha256(key.encode()).digest()[:8], "little")
    inters, reps, _ = schedule_joint(tg, int(nbits), seed=seed) if int(nbits) > 8 else schedule(tg)
    return key, ([[int(w), [int(o) for o in ops]] for w, ops in inters], {str(t): list(r) for t, r in reps.items()})


def window_cost(targets):
    """Op count of the reference-style window tables (what the generator emitted before)."""
    have = set()
    ops = 0
    for v in targets:
        if not v:
            continue
        ops += 1
        for h, n in ((0, v & 15), (1, v >> 4)):
            if n and bin(n).count("1") > 1:
                have.add((h, n))
    for h in (0, 1):
        if (h, 15) in have:
            for s in (3, 12):
                have.add((h, s))
    return ops + len(have)


if __name__ == "__main__":
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import time
    from gen_fixed_kernels import generator, row_bytes
    k, m = (int(a) for a in (sys.argv[1:3] if len(sys.argv) > 2 else (200, 32)))
    rows = generator(k, m)
    t0 = time.time()
    old = new = n = 0
    for p in range(0, m, 8):
        for x in range(k):
            tg = [v for y in range(p, min(m, p + 8)) for v in row_bytes(rows[y][x])]
            old += window_cost(tg)
            new += schedule(tg)[2]
            n += 1
    print(f"({k},{m}) part-steps={n} window={old / n:.2f} slp={new / n:.2f} ops/part-step "
          f"({new / old:.3f}) {time.time() - t0:.1f}s")
