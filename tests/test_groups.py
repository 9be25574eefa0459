"""Packet-group framing (include/shorthair_groups.h).

The GPU path (shorthair_amd.groups -> libcauchy256 shorthair_encode_groups /
shorthair_recover_groups) is compared byte for byte with oracle/packets.py, a per-group
restatement of the reference's EncodeQueued + GenerateRecoveryBlock and RecoverGroup
(Shorthair.cpp:480-609, :704-761) on the C oracle codec; the codec bytes themselves are pinned by
tests/golden. Edge cases follow the reference's: k == 1 special form, k + m > 256 truncation,
m == 1, zero-length and maximum-size payloads, groups that cannot be or need not be decoded,
malformed receiver input.
"""
import random

import numpy as np
import pytest

from oracle import packets as opk
from oracle import pyoracle as po


@pytest.fixture(scope="module")
def ora():
    return po.oracle()


def _payloads(rng, k, largest):
    return [bytes(rng.getrandbits(8) for _ in range(rng.randint(0, largest))) for _ in range(k)]


def _fast_payloads(nprng, k, largest, lo=0):
    lens = nprng.integers(lo, largest + 1, size=k)
    return [nprng.integers(0, 256, size=int(n), dtype=np.uint8).tobytes() for n in lens]


def _lose(rng, k, packets, recovery, n_lost, n_rec):
    """Arrival lists after losing n_lost originals; n_rec recovery packets arrive (shuffled)."""
    lost = set(rng.sample(range(k), n_lost))
    orig = [(i, packets[i]) for i in range(k) if i not in lost]
    rng.shuffle(orig)
    rec = rng.sample(recovery, min(n_rec, len(recovery)))
    return lost, orig, rec


# ---------------------------------------------------------------- CPU: the restatement itself

@pytest.mark.parametrize("k,m", [(2, 1), (5, 3), (20, 9), (60, 40), (250, 10)])
def test_oracle_framing_round_trip(ora, k, m):
    rng = random.Random(k * 1000 + m)
    pk = _payloads(rng, k, 90)
    rec = opk.tx_group(ora, m, pk)
    mm = min(m, 256 - k)
    assert len(rec) == mm
    B = opk.roundup8(2 + max(len(p) for p in pk))
    assert all(len(r) == 3 + B and r[1] == k - 1 and r[2] == mm - 1 for r in rec)
    assert [r[0] for r in rec] == list(range(k, k + mm))
    e = min(mm, k)
    lost, orig, got = _lose(rng, k, pk, rec, e, e)
    out = opk.rx_group(ora, orig, got)
    assert sorted(i for i, _ in out) == sorted(lost)
    assert all(pk[i] == p for i, p in out)
    assert [i for i, _ in out] == sorted(lost)  # i-th recovery block <- i-th smallest erasure


def test_oracle_framing_special_cases(ora):
    assert opk.tx_group(ora, 0, [b"x"]) is None  # m < 1
    assert opk.tx_group(ora, 3, [b"ab"]) == [b"\x01\x00ab"] * 3  # k == 1
    assert opk.rx_group(ora, [], [b"\x01\x00ab"]) == [(0, b"ab")]
    assert opk.rx_group(ora, [(0, b"ab")], [b"\x01\x00ab"]) is None


# ---------------------------------------------------------------- CPU: boundary without a GPU

def test_recovery_packet_bytes_without_gpu():
    from shorthair_amd import groups as sg
    assert sg.recovery_packet_bytes(1, [17]) == 19
    assert sg.recovery_packet_bytes(3, [1, 6, 5]) == 3 + 8
    assert sg.recovery_packet_bytes(3, [1, 7, 5]) == 3 + 16
    assert sg.recovery_packet_bytes(0, []) == -1
    assert sg.recovery_packet_bytes(256, [1] * 256) == -1


@pytest.mark.parametrize("bad", [[(0, [b"a", b"b"])], [(2, [])], [(2, [b"a"] * 256)]])
def test_encode_groups_rejects_invalid_without_gpu(bad):
    from shorthair_amd import groups as sg
    with pytest.raises(ValueError):
        sg.encode_groups(bad)


@pytest.mark.parametrize("bad", [
    [([(5, b"a")], [bytes([2, 1, 1]) + bytes(8)])],                # original id >= k (k = 2)
    [([(0, b"a"), (0, b"b")], [bytes([3, 2, 1]) + bytes(8)])],     # duplicate id (k = 3)
    [([(0, b"a")], [bytes([2, 1, 1]) + bytes(7)])],                # block bytes not a multiple of 8
    [([(0, bytes(7))], [bytes([2, 1, 1]) + bytes(8)])],            # payload longer than B - 2
    [([(0, b"a")], [bytes([1, 1, 1]) + bytes(8)])],                # recovery id < k
    [([(0, b"a")], [bytes([2, 1, 1]) + bytes(8), bytes([3, 2, 1]) + bytes(8)])],  # k disagrees
])
def test_recover_groups_rejects_malformed_without_gpu(bad):
    from shorthair_amd import groups as sg
    with pytest.raises(ValueError):
        sg.recover_groups(bad)


def test_recover_groups_skips_undecodable_without_gpu():
    """Nothing to decode -> no GPU touched, no callback (CanRecover() false / all seen)."""
    from shorthair_amd import groups as sg
    rec = bytes([3, 2, 1]) + bytes(8)
    assert sg.recover_groups([([(0, b"a")], [rec])]) == (0, [])                      # 2 < k = 3
    assert sg.recover_groups([([(0, b"a"), (1, b""), (2, b"c")], [rec])]) == (0, [])  # all seen
    assert sg.recover_groups([([(0, b"a")], [])]) == (0, [])                          # no recovery
    assert sg.recover_groups([([], [b"\x01\x00hello"])]) == (1, [(0, 0, b"hello")])   # k == 1


# ---------------------------------------------------------------- GPU parity

def _mixed_groups(seed, n):
    rng = random.Random(seed)
    nprng = np.random.default_rng(seed)
    shapes = [(1, 4), (2, 1), (3, 2), (9, 1), (16, 5), (20, 9), (64, 16), (100, 200), (200, 32),
              (250, 9), (255, 3)]
    out = []
    for i in range(n):
        k, m = shapes[i % len(shapes)]
        largest = rng.choice([0, 1, 6, 14, 175, 1398]) if k > 1 else rng.randint(0, 300)
        pk = _fast_payloads(nprng, k, largest)
        if largest and k > 1:
            pk[rng.randrange(k)] = nprng.integers(0, 256, size=largest, dtype=np.uint8).tobytes()
        out.append((m, pk))
    return out


@pytest.mark.gpu
def test_encode_groups_matches_reference_framing(ora):
    from shorthair_amd import groups as sg
    groups = _mixed_groups(11, 44)
    got = sg.encode_groups(groups)
    for (m, pk), rec in zip(groups, got):
        assert rec == opk.tx_group(ora, m, pk)


@pytest.mark.gpu
def test_recover_groups_matches_reference_delivery(ora):
    from shorthair_amd import groups as sg
    groups = _mixed_groups(12, 44)
    recs = sg.encode_groups(groups)
    rng = random.Random(5)
    rx, expect, lost_sets = [], [], []
    for gi, ((m, pk), rec) in enumerate(zip(groups, recs)):
        k = len(pk)
        mm = len(rec)
        if k == 1:
            lost, orig, got = {0}, [], rec[:1]
        else:
            e = rng.randint(1, min(k, mm))
            lost, orig, got = _lose(rng, k, pk, rec, e, rng.randint(e, mm))
        rx.append((orig, got))
        expect.append(opk.rx_group(ora, orig, got))
        lost_sets.append(lost)
    n, delivered = sg.recover_groups(rx)
    assert n == len(groups)
    by_group = {}
    for g, pid, p in delivered:
        by_group.setdefault(g, []).append((pid, p))
    for gi, (m, pk) in enumerate(groups):
        assert by_group.get(gi) == expect[gi], gi
        assert sorted(i for i, _ in by_group[gi]) == sorted(lost_sets[gi])
        assert all(pk[i] == p for i, p in by_group[gi])


@pytest.mark.gpu
def test_groups_multi_chunk_headline_shape(ora):
    """k=200, m=32, 1398-byte payloads: 400 groups span several double-buffered chunks; every
    group loses 32 originals (worst case), all recovered; a sample checked against the oracle."""
    from shorthair_amd import groups as sg
    nprng = np.random.default_rng(3)
    G, k, m = 400, 200, 32
    groups = [(m, _fast_payloads(nprng, k, 1398, lo=1000)) for _ in range(G)]
    for _, pk in groups:
        pk[0] = nprng.integers(0, 256, size=1398, dtype=np.uint8).tobytes()  # B = 1400
    recs = sg.encode_groups(groups)
    assert all(len(r) == m and len(r[0]) == 1403 for r in recs)
    for gi in (0, 177, G - 1):
        assert recs[gi] == opk.tx_group(ora, m, groups[gi][1])
    rng = random.Random(9)
    rx, lost_sets = [], []
    for (_, pk), rec in zip(groups, recs):
        lost, orig, got = _lose(rng, k, pk, rec, m, m)
        rx.append((orig, got))
        lost_sets.append(lost)
    n, delivered = sg.recover_groups(rx)
    assert n == G and len(delivered) == G * m
    for g, pid, p in delivered:
        assert pid in lost_sets[g] and groups[g][1][pid] == p
    sample = [d for d in delivered if d[0] == 123]
    assert [(pid, p) for _, pid, p in sample] == opk.rx_group(ora, *rx[123])


@pytest.mark.gpu
def test_groups_concurrent_calls(ora):
    """Two threads frame and recover packet groups at once: a framing pass that finds
    the host worker pool busy runs on its own thread, so both calls progress; every result exact."""
    import threading
    from shorthair_amd import groups as sg
    errors = []

    def worker(seed):
        try:
            groups = _mixed_groups(seed, 33)
            for _ in range(3):
                recs = sg.encode_groups(groups)
                for (m, pk), rec in zip(groups, recs):
                    assert rec == opk.tx_group(ora, m, pk)
                rng = random.Random(seed)
                rx, lost_sets = [], []
                for (m, pk), rec in zip(groups, recs):
                    k = len(pk)
                    if k == 1:
                        lost, orig, got = {0}, [], rec[:1]
                    else:
                        e = rng.randint(1, min(k, len(rec)))
                        lost, orig, got = _lose(rng, k, pk, rec, e, e)
                    rx.append((orig, got))
                    lost_sets.append(lost)
                n, delivered = sg.recover_groups(rx)
                assert n == len(groups)
                for g, pid, p in delivered:
                    assert pid in lost_sets[g] and groups[g][1][pid] == p
                assert len(delivered) == sum(len(s) for s in lost_sets)
        except Exception as ex:  # reported on the main thread
            errors.append((seed, repr(ex)))

    threads = [threading.Thread(target=worker, args=(s,)) for s in (31, 32)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=120)
    assert not any(th.is_alive() for th in threads)
    assert not errors, errors
