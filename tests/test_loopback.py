"""Deterministic fake-clock loopback (shorthair_amd/loopback.py).

The reference's only end-to-end check is tests/Tester.cpp's ZeroLossTest, a wall-clock loop that
never exits (:224-240). The loopback restates it on a counter, so a run is reproducible: the
same arguments give the same code groups, losses and deliveries. On the CPU the driver runs on
the oracle's framing (oracle/packets.py over the C oracle codec) to check the driver itself;
on the GPU it drives the batched framing API and must reproduce the oracle run exactly.
"""
import numpy as np
import pytest

from shorthair_amd import loopback as lb


class OracleCodec:
    """shorthair_amd.groups' two calls on the per-group CPU restatement (test infrastructure)."""

    def __init__(self):
        from oracle import pyoracle as po
        self.ora = po.oracle()

    def encode_groups(self, groups):
        from oracle import packets as opk
        return [opk.tx_group(self.ora, m, pk) for m, pk in groups]

    def recover_groups(self, groups):
        from oracle import packets as opk
        n, out = 0, []
        for g, (orig, rec) in enumerate(groups):
            got = opk.rx_group(self.ora, orig, rec)
            if got is not None:
                n += 1
                out += [(g, pid, p) for pid, p in got]
        return n, out


def test_pcg_matches_oracle_generator():
    """SiameseTools.h:80-102 PCGRandom: the loopback's generator against the C oracle's
    (ora_fill_block(0, x, 0) emits PCG(x) four bytes per draw, the loopback the low byte)."""
    from oracle import pyoracle as po
    blocks = po.fill_group(0, 40, 4 * 64, 0)
    got = lb.pcg_bytes(list(range(40)), 64)
    assert np.array_equal(got, blocks[:, ::4])
    p = lb.PCG(7)
    assert [p.next() & 0xFF for _ in range(64)] == list(lb.pcg_bytes([7], 64)[0])


def test_redundancy_policy_gives_tester_shapes():
    """ShorthairCodec::Tick at the estimator's floor (0.03): R = 1.2 N, truncated to 256 - k."""
    assert lb.recovery_count(200, 0.03) == 240 and lb.recovery_count(190, 0.03) == 228
    assert lb.recovery_count(2, 0.03) == 2 and lb.recovery_count(10, 0.03) == 12
    # the approximation branch (N*plr >= 10): never more than 1.5N + 1
    for n in (100, 200, 400):
        r = lb.recovery_count(n, 0.1)
        assert int(0.2 * n) <= r <= int(1.5 * n) + 1


def test_loopback_driver_on_oracle_is_deterministic():
    """~12 code groups of the Tester's shapes through the oracle framing: every decodable
    group's missing originals are delivered with the sender's bytes, the accounting closes,
    and a second run gives identical results."""
    a = lb.run(240, codec=OracleCodec(), batch=4)
    assert a.bad == [], a.bad[:3]
    assert a.groups >= 10 and a.recovered == a.expected_recovered > 0
    assert a.received + a.lost == a.sent
    assert {k for (k, m, _) in a.shapes} <= {190, 200} and all(k + m == 256 for (k, m, _) in a.shapes)
    b = lb.run(240, codec=OracleCodec(), batch=4)
    assert vars(a) == vars(b)


def test_loopback_heavy_loss_leaves_undecodable_groups():
    """At 30 % channel loss some groups get fewer than k packets: those originals are lost,
    never delivered wrong."""
    st = lb.run(120, loss=0.3, codec=OracleCodec(), batch=3)
    assert st.bad == [] and st.lost > 0 and st.recovered == st.expected_recovered


@pytest.mark.gpu
def test_loopback_gpu_reproduces_oracle_run():
    """The same loopback on the GPU framing API (batched encode / decode): identical statistics
    to the oracle run, every recovered payload checked against PCG(id)."""
    gpu = lb.run(400, batch=8)
    assert gpu.bad == [], gpu.bad[:3]
    assert gpu.recovered == gpu.expected_recovered > 0
    assert {(k, m) for (k, m, _) in gpu.shapes} == {(200, 56), (190, 66)}
    ora = lb.run(400, batch=8, codec=OracleCodec())
    assert vars(gpu) == vars(ora)
