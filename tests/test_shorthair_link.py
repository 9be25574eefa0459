"""The reference's unchanged caller on our library (VERDICT r2 "missing #4"): catid/shorthair's
protocol layer (Shorthair.cpp, PacketAllocator.cpp, SiameseTools.cpp, compiled from
/root/reference by oracle/Makefile) linked against shorthair_amd/libcauchy256.so and driven by a
Tester-shaped loopback (oracle/shorthair_link.cpp: 10 packets of 8..1350 bytes per 5 ms tick, 10 %
wire loss). Every delivered payload is checked byte for byte inside the harness."""
import json
import os
import subprocess

import pytest

ROOT = os.path.normpath(os.path.join(os.path.dirname(__file__), ".."))
EXE = os.path.join(ROOT, "oracle", "_ref", "shorthair_link")


def test_link_binary_uses_only_the_reference_abi():
    """The linked caller needs exactly the three cauchy_256.h entry points from the codec."""
    if not os.path.exists(EXE):
        pytest.skip("oracle/_ref/shorthair_link not built (needs /root/reference at build time)")
    out = subprocess.run(["nm", "-u", EXE], capture_output=True, text=True, check=True).stdout
    codec = sorted(l.split()[-1] for l in out.splitlines() if "cauchy" in l or "gf256" in l)
    assert codec == ["_cauchy_256_init", "cauchy_256_decode", "cauchy_256_encode"]


@pytest.mark.gpu
def test_reference_shorthair_loopback_on_gpu_codec():
    if not os.path.exists(EXE):
        pytest.skip("oracle/_ref/shorthair_link not built (needs /root/reference at build time)")
    res = subprocess.run([EXE, "--seconds", "3"], capture_output=True, text=True, timeout=120)
    line = [l for l in res.stdout.splitlines() if l.startswith("{")][-1]
    r = json.loads(line)
    assert res.returncode == 0, (res.returncode, res.stderr[-2000:])
    assert r["corrupt"] == 0 and r["duplicate"] == 0, r
    assert r["sent"] > 1000 and r["wire_dropped"] > 50, r
    # 10 % of the wire packets are dropped; FEC must recover nearly all lost originals (the
    # reference's Tester reaches ~0.998 on its own codec)
    assert r["delivery_ratio"] >= 0.99, r
