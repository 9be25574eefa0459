"""CPU checks of bench.py's host-side legs (no GPU): the CPU baseline runs the reference build
and reports the contract's fields; the PMC traffic lookup refuses a summary of another build."""
import os

import pytest

ROOT = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def test_cpu_baseline_runs_reference():
    import bench
    if not os.path.exists(os.path.join(ROOT, "oracle", "_ref", "libref_cauchy.so")):
        pytest.skip("oracle/_ref not built")
    cpu = bench.cpu_baseline(28, 4, 1400, 0, 0.2, 2)
    assert cpu is not None and cpu["kind"] == "reference" and cpu["cores"] == 2
    assert cpu["value"] > 0 and cpu["unit"] == "GiB/s" and "group pairs" in cpu["sample"]


def test_traffic_lookup_requires_matching_build():
    import bench
    import shorthair_amd as sh

    class Fake:
        LIB_PATH = os.path.join(ROOT, "bench.py")  # any file whose hash no summary carries

    assert bench.pmc_traffic(Fake, "dec", 200, 32, 1400, 8192, 32) == (None, None)
    t, src = bench.pmc_traffic(sh, "dec", 200, 32, 1400, 8192, 32)
    assert (t is None) == (src is None)
