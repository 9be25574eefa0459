"""CPU checks of the kernel generator (tools/gen_fixed_kernels.py): the column snippets of the
tile kernels' decode stage A index a 4-row coefficient block by the input's Cauchy parameter X'_x
alone, which holds only because the rows' Y' are the same for every m >= 7 (reference
cauchy_matrix(), cauchy_256.cpp:453-477)."""
import importlib.util
import os

import pytest

ROOT = os.path.normpath(os.path.join(os.path.dirname(__file__), ".."))


def _gen():
    spec = importlib.util.spec_from_file_location("gen_fixed_kernels", os.path.join(ROOT, "tools", "gen_fixed_kernels.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.parametrize("k,m", [(150, 40), (180, 76), (120, 136), (50, 10), (200, 32), (2, 254), (249, 7), (90, 49)])
def test_column_coefficients_match_generator(k, m):
    g = _gen()
    G = g.generator(k, m)
    xp = g.cauchy_xp(k, m)
    for y in range(m):
        for x in range(k):
            assert g.col_coef(y, xp[x]) == G[y][x], (y, x)


def test_generator_matches_reference_goldens_shape():
    """The Python generator restates the same table bytes the library ships: row 0 is all ones and
    every coefficient of an m >= 7 generator is non-zero (an MDS Cauchy matrix)."""
    g = _gen()
    G = g.generator(64, 16)
    assert G[0] == [1] * 64
    assert all(c != 0 for row in G for c in row)


def test_part_layouts_fill_the_simds():
    """Every compile-time shape's workgroup has a multiple of 4 waves."""
    g = _gen()
    for k, m in g.CONFIGS:
        P, CW, R, minw, sync = g.shape(k, m)
        assert (P * CW) % 4 == 0, (k, m, P, CW)
        assert R >= 2 * sync + 1 and R * 8 * CW * 64 * 4 <= 131072
        assert (m + P - 1) // P <= 9


def _symbolic_run(lines, k, nr, x0=0):
    """Evaluate a generated part body symbolically: every 32-bit word is the XOR of a set of input
    sub-blocks, held as an int bitmask (bit 8x + a = sub-block a of input block x). Returns the
    accumulators [nr][8]. Reads follow the body's src.read(slot, ...) calls in order: the i-th read
    loads input block i (encode steps are the input blocks in order)."""
    import re
    env, acc, nread = {}, [[0] * 8 for _ in range(nr)], 0

    def val(tok):
        tok = tok.strip()
        m = re.fullmatch(r"acc\[(\d+)\]\[(\d+)\]", tok)
        return acc[int(m.group(1))][int(m.group(2))] if m else env[tok]

    for ln in lines:
        ln = ln.strip()
        m = re.match(r"src\.read\((\d+), (.*)\);", ln)
        if m:
            for a, w in enumerate(m.group(2).split(",")):
                env[w.strip()] = 1 << (8 * (x0 + nread) + a)
            nread += 1
            continue
        m = re.match(r"const uint32_t (\w+) = X3\((\w+), (\w+), (\w+)\);", ln)
        if m:
            env[m.group(1)] = val(m.group(2)) ^ val(m.group(3)) ^ val(m.group(4))
            continue
        m = re.match(r"const uint32_t (\w+) = (\w+) \^ (\w+);", ln)
        if m:
            env[m.group(1)] = val(m.group(2)) ^ val(m.group(3))
            continue
        m = re.match(r"acc\[(\d+)\]\[(\d+)\] = X3\(acc\[\1\]\[\2\], (\w+), (\w+)\);", ln)
        if m:
            acc[int(m.group(1))][int(m.group(2))] ^= val(m.group(3)) ^ val(m.group(4))
            continue
        m = re.match(r"XV\(acc\[(\d+)\]\[(\d+)\], (\w+)\);", ln)
        if m:
            acc[int(m.group(1))][int(m.group(2))] ^= val(m.group(3))
    assert nread == k
    return acc


@pytest.mark.parametrize("k,m,joint", [(20, 16, 2), (20, 16, 1), (9, 12, 2), (28, 4, 2)])
def test_scheduled_xor_programs_compute_the_bitmatrix(k, m, joint, monkeypatch):
    """The straight-line XOR programs the generator emits (tools/xor_sched.py units of one or two
    input blocks) compute exactly the reference's bitmatrix product: output sub-block b of row y
    = XOR over inputs x and bits a of C[y][x] * 2^b of input sub-block a (cauchy_256.cpp:1398-1477
    semantics), for every part of the row split."""
    g = _gen()
    monkeypatch.setattr(g, "JOINT", joint)
    rows = g.generator(k, m)
    steps = [("c", x) for x in range(k)]
    for y0, y1 in ((0, min(m, 8)), (8, min(m, 16))):
        if y0 >= m:
            continue
        body = g.Body(k, rows, y0, y1)
        body.emit(16, 4, steps, (k + 3) & ~3)
        acc = _symbolic_run(body.lines, k, y1 - y0)
        for yi in range(y1 - y0):
            for b in range(8):
                want = sum(g.row_bytes(rows[y0 + yi][x])[b] << (8 * x) for x in range(k))
                assert acc[yi][b] == want, (y0 + yi, b)


@pytest.mark.parametrize("k,m", [(20, 16), (28, 4), (200, 32)])
def test_split_tile_halves_sum_to_the_product(k, m):
    """Split tiles (fixed_common.hpp RowSink "Split tiles"): the two half-step programs the
    generator emits (steps cut at an even index, as gen_config does) compute partial products that
    XOR to the whole bitmatrix product -- what the second arriving workgroup stores."""
    g = _gen()
    rows = g.generator(k, m)
    steps = [("c", x) for x in range(k)]
    n0 = (len(steps) // 2) & ~1
    y0, y1 = 0, min(m, 8)
    parts = []
    for sub, x0 in ((steps[:n0], 0), (steps[n0:], n0)):
        body = g.Body(k, rows, y0, y1)
        body.emit(16, 4, sub, (k + 3) & ~3)
        parts.append(_symbolic_run(body.lines, len(sub), y1 - y0, x0))
    for yi in range(y1 - y0):
        for b in range(8):
            want = sum(g.row_bytes(rows[y0 + yi][x])[b] << (8 * x) for x in range(k))
            assert parts[0][yi][b] ^ parts[1][yi][b] == want, (yi, b)
            assert parts[0][yi][b] >> (8 * n0) == 0  # half 0 touches blocks < n0 only
