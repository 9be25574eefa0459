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
