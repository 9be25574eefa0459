"""GPU parity tests: the HIP path (through the C ABI) against the reference's golden vectors, the
oracle, and size-independent properties at BASELINE.json's full sizes. Bit-exact everywhere
(integer/byte arithmetic: no tolerance)."""
import ctypes

import numpy as np
import pytest

from oracle import pyoracle as po
from tests.golden_util import case_inputs, manifest, sha, vectors

pytestmark = pytest.mark.gpu
CASES = manifest()


@pytest.fixture(scope="module")
def sh():
    import torch
    import shorthair_amd
    assert shorthair_amd.cauchy_256_init() == 0
    torch.cuda.init()
    return shorthair_amd


def _dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _sync():
    import torch
    torch.cuda.synchronize()


# ------------------------------------------------------------------------- golden vectors
@pytest.mark.parametrize("c", [c for c in CASES if c["kind"] == "encode"], ids=lambda c: c["name"])
def test_encode_batch_golden(sh, c):
    import torch
    k, m, B = c["k"], c["m"], c["B"]
    data, _ = case_inputs(po, c)
    d_in = _dev(data[None])
    d_out = torch.zeros((1, m, B), dtype=torch.uint8, device="cuda")
    rc = sh.encode_batch(k, m, B, 1, d_in, d_out)
    _sync()
    assert rc == c["rc"]
    out = d_out[0].cpu().numpy()
    assert sha(out) == c["out_sha"]
    if c["full"]:
        assert np.array_equal(out, vectors()[c["name"] + "_out"])


@pytest.mark.parametrize("c", [c for c in CASES if c["kind"] == "decode"], ids=lambda c: c["name"])
def test_decode_batch_golden(sh, c):
    k, m, B = c["k"], c["m"], c["B"]
    data, rows = case_inputs(po, c)
    _, rec = po.oracle().encode(k, m, data, B)
    whole = np.concatenate([data, rec])
    blocks = np.stack([whole[r] for r in rows])
    assert sha(blocks) == c["in_sha"]
    d_blocks, d_rows = _dev(blocks[None]), _dev(rows[None])
    rc = sh.decode_batch(k, m, B, 1, d_blocks, d_rows)
    _sync()
    assert rc == c["rc"]
    assert d_rows[0].cpu().numpy().tolist() == c["rows_out"]
    out = d_blocks[0].cpu().numpy()
    assert sha(out) == c["out_sha"]
    if c["full"]:
        assert np.array_equal(out, vectors()[c["name"] + "_out"])


# ------------------------------------------------------------------------- drop-in single-group ABI
@pytest.mark.parametrize("c", [c for c in CASES if c["kind"] == "encode" and c["full"]],
                         ids=lambda c: c["name"])
def test_single_group_encode_abi_misaligned(sh, c):
    """cauchy_256_encode on host pointers misaligned like Shorthair's (p->data + 3)."""
    k, m, B = c["k"], c["m"], c["B"]
    data, _ = case_inputs(po, c)
    raw = np.zeros(k * (B + 16) + 64, np.uint8)
    ptrs = []
    for x in range(k):
        off = 3 + x * (B + 16)
        raw[off:off + B] = data[x]
        ptrs.append(raw.ctypes.data + off)
    rec_raw = np.zeros(m * B + 8, np.uint8)
    rc = sh.cauchy_256_encode(k, m, ptrs, rec_raw.ctypes.data + 5, B)
    assert rc == c["rc"]
    out = rec_raw[5:5 + m * B].reshape(m, B)
    assert np.array_equal(out, vectors()[c["name"] + "_out"])


@pytest.mark.parametrize("c", [c for c in CASES if c["kind"] == "decode" and c["full"]],
                         ids=lambda c: c["name"])
def test_single_group_decode_abi(sh, c):
    k, m, B = c["k"], c["m"], c["B"]
    data, rows = case_inputs(po, c)
    _, rec = po.oracle().encode(k, m, data, B)
    whole = np.concatenate([data, rec])
    bufs = [np.concatenate([np.zeros(1, np.uint8), whole[r]]) for r in rows]  # +1 misalign
    arr = (sh.Block * k)()
    for i in range(k):
        arr[i].data = bufs[i].ctypes.data + 1
        arr[i].row = int(rows[i])
    rc = sh.cauchy_256_decode(k, m, arr, B)
    assert rc == c["rc"]
    assert [arr[i].row for i in range(k)] == c["rows_out"]
    out = np.stack([b[1:] for b in bufs])
    assert np.array_equal(out, vectors()[c["name"] + "_out"])


# m >= 7: host-side setup; m in {2, 4, 5, 6}: the device setup (Gauss-Jordan over the searched
# tables) writing into the staging workspace, rows placed by the host; B = 1000 and
# 520 are no compile-time shape (tile kernels), B = 96 is below the tile kernels (generic path).
@pytest.mark.parametrize("k,m,B", [(200, 32, 1400), (64, 16, 1400), (150, 40, 1352), (28, 8, 256),
                                   (100, 20, 512), (190, 66, 1336), (12, 7, 64),
                                   (20, 2, 1400), (28, 4, 256), (40, 6, 1000), (30, 4, 96), (17, 5, 520),
                                   # k below a compiled K of the same m (fixed_kernel_k)
                                   (150, 32, 1400), (20, 4, 256), (130, 56, 1352), (150, 40, 1400)])
def test_single_group_decode_random_patterns(sh, k, m, B):
    """cauchy_256_decode (host-side setup for m >= 7) on random erasure sets: e = 1..min(k, m) lost
    originals, a random subset of e recovery rows, blocks in random array order; results and rows
    against the oracle's decode of the same array."""
    ora = po.oracle()
    rng = np.random.default_rng(k * 1000 + m)
    data = po.fill_group(k + m, k, B, 0x5A)
    rc, rec = ora.encode(k, m, data, B)
    assert rc == 0
    whole = np.concatenate([data, rec])
    for trial in range(6):
        e = int(rng.integers(1, min(k, m) + 1)) if trial else min(k, m)
        lost = rng.choice(k, size=e, replace=False)
        recv = k + rng.choice(m, size=e, replace=False)
        rows = np.array(sorted(set(range(k)) - set(lost.tolist())) + recv.tolist())
        rng.shuffle(rows)
        bufs = [whole[r].copy() for r in rows]
        ref = [whole[r].copy() for r in rows]
        rc_ref, rows_ref = ora.decode(k, m, ref, rows.tolist(), B)
        arr = (sh.Block * k)(*[sh.Block(b.ctypes.data, int(r)) for b, r in zip(bufs, rows)])
        assert sh.cauchy_256_decode(k, m, arr, B) == rc_ref == 0
        assert [arr[i].row for i in range(k)] == rows_ref
        for i in range(k):
            assert np.array_equal(bufs[i], ref[i]), (trial, i)
            assert np.array_equal(bufs[i], data[rows_ref[i]])


def test_single_group_abi_concurrent(sh):
    """Single-group calls from several threads at once (two Shorthair codec objects on two threads):
    each call holds its own staging slot and stream, so the calls overlap and none sees another's
    data. Every result is checked against the oracle."""
    import threading
    ora = po.oracle()
    shapes = [(200, 32, 1400), (64, 16, 1400), (28, 4, 256), (12, 5, 64), (150, 40, 1352), (2, 2, 8)]
    jobs = []
    for t, (k, m, B) in enumerate(shapes):
        data = po.fill_group(900 + t, k, B, 0x77)
        rc, rec = ora.encode(k, m, data, B)
        assert rc == 0
        e = min(m, k)
        rows = np.array(list(range(e, k)) + list(range(k, k + e)), np.uint8)
        jobs.append((k, m, B, data, rec, rows))
    errors = []

    def worker(job, iters=12):
        k, m, B, data, rec, rows = job
        whole = np.concatenate([data, rec])
        try:
            for _ in range(iters):
                out = np.zeros(m * B, np.uint8)
                assert sh.cauchy_256_encode(k, m, [data[x].ctypes.data for x in range(k)], out.ctypes.data, B) == 0
                assert np.array_equal(out.reshape(m, B), rec)
                bufs = [whole[r].copy() for r in rows]
                arr = (sh.Block * k)(*[sh.Block(b.ctypes.data, int(r)) for b, r in zip(bufs, rows)])
                assert sh.cauchy_256_decode(k, m, arr, B) == 0
                for i in range(k):
                    assert np.array_equal(bufs[i], data[arr[i].row])
        except Exception as ex:  # reported on the main thread
            errors.append((k, m, B, repr(ex)))

    threads = [threading.Thread(target=worker, args=(j,)) for j in jobs for _ in range(2)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=120)
    assert not any(th.is_alive() for th in threads)
    assert not errors, errors


# ------------------------------------------------------------------------- batches vs oracle
def _oracle_encode_groups(k, m, B, cfg, groups):
    ora = po.oracle()
    res = {}
    for g in groups:
        data = po.fill_group(g, k, B, cfg)
        rc, out = ora.encode(k, m, data, B)
        assert rc == 0
        res[g] = (data, out)
    return res


@pytest.mark.parametrize("k,m,B,G", [(64, 16, 1400, 4096), (28, 4, 256, 512), (112, 16, 1400, 300),
                                     (224, 32, 65536, 8), (200, 32, 1400, 1024), (2, 2, 8, 1000),
                                     (250, 6, 16, 64), (13, 9, 24, 333),
                                     # k below a compiled K of the same m: the kernel's steps past
                                     # k read zeros (fixed_kernel_k)
                                     (150, 32, 1400, 300), (100, 16, 1400, 300), (20, 4, 1400, 500),
                                     (150, 56, 1352, 100), (120, 66, 1336, 100), (40, 16, 264, 700),
                                     (135, 32, 256, 900), (150, 40, 1400, 301), (216, 40, 1400, 64)])
def test_encode_batch_vs_oracle(sh, k, m, B, G):
    """BASELINE configs[1] (4096 x k=64 m=16 1400B) and sweep shapes: device-generated input
    equals the oracle's generator (sha of a sample), encode bit-exact on sampled groups."""
    import torch
    cfg = 0xC2 + k
    d_in = torch.empty((G, k, B), dtype=torch.uint8, device="cuda")
    d_out = torch.empty((G, m, B), dtype=torch.uint8, device="cuda")
    assert sh.fill_synthetic(d_in, k, B, G, 0, cfg) == 0
    assert sh.encode_batch(k, m, B, G, d_in, d_out) == 0
    _sync()
    sample = sorted({0, 1, G // 2, G - 2, G - 1})
    exp = _oracle_encode_groups(k, m, B, cfg, sample)
    for g in sample:
        assert np.array_equal(d_in[g].cpu().numpy(), exp[g][0]), f"input g={g}"
        assert np.array_equal(d_out[g].cpu().numpy(), exp[g][1]), f"recovery g={g}"


def test_encode_manifest_big_shapes(sh):
    """Digests of the reference on the C2/C3/C4 shapes (tests/golden/manifest.json big_enc_*)."""
    import torch
    for c in [c for c in CASES if c["kind"] == "encode" and c["name"].startswith("big_")]:
        k, m, B = c["k"], c["m"], c["B"]
        d_in = torch.empty((1, k, B), dtype=torch.uint8, device="cuda")
        d_out = torch.empty((1, m, B), dtype=torch.uint8, device="cuda")
        sh.fill_synthetic(d_in, k, B, 1, c["g"], c["cfg"])
        assert sh.encode_batch(k, m, B, 1, d_in, d_out) == 0
        _sync()
        assert sha(d_in[0].cpu().numpy()) == c["in_sha"], c["name"]
        assert sha(d_out[0].cpu().numpy()) == c["out_sha"], c["name"]


def _decode_inputs(k, m, B, G, cfg, e_fixed):
    """Device-resident decode batch: encode on the GPU, then gather each group's received blocks
    in the order of its (oracle-generated) erasure pattern."""
    import torch
    data = torch.empty((G, k, B), dtype=torch.uint8, device="cuda")
    rec = torch.empty((G, m, B), dtype=torch.uint8, device="cuda")
    assert __import__("shorthair_amd").fill_synthetic(data, k, B, G, 0, cfg) == 0
    assert __import__("shorthair_amd").encode_batch(k, m, B, G, data, rec) == 0
    rows = np.zeros((G, k), np.uint8)
    es = np.zeros(G, np.int64)
    for g in range(G):
        es[g], rows[g] = po.erasure_pattern(g, k, m, cfg, e_fixed)
    d_rows = torch.from_numpy(rows).cuda()
    whole = torch.cat([data, rec], dim=1)
    idx = d_rows.long()
    blocks = whole[torch.arange(G, device="cuda")[:, None], idx].contiguous()
    del whole
    return data, rec, blocks, d_rows, rows, es


@pytest.mark.parametrize("k,m,B,G,e_fixed", [(200, 32, 1400, 8192, 0), (200, 32, 1400, 2048, 32),
                                             (64, 16, 1400, 1024, 0), (28, 4, 256, 700, 0),
                                             (112, 16, 65536, 6, 0), (128, 128, 8, 64, 0),
                                             (30, 9, 48, 500, 9),
                                             # e = m on the searched tables (two Gauss-Jordan
                                             # elements per lane at e = 6)
                                             (20, 6, 1400, 999, 6), (12, 5, 64, 300, 5),
                                             (40, 6, 256, 513, 0),
                                             # small blocks on the compile-time path (stageb_small,
                                             # nq = 4 / 8 / 12 / 16 word columns, shifted chunks)
                                             (28, 4, 128, 3001, 0), (224, 32, 256, 601, 0),
                                             (112, 16, 384, 333, 16), (200, 32, 136, 257, 0),
                                             (200, 56, 512, 129, 0), (64, 16, 264, 77, 0),
                                             # k below a compiled K of the same m
                                             (150, 32, 1400, 500, 0), (100, 16, 1400, 500, 16),
                                             (20, 4, 256, 3000, 0), (150, 56, 1352, 200, 0),
                                             (120, 66, 1336, 200, 0), (40, 16, 256, 2000, 0),
                                             (150, 40, 1400, 301, 0), (216, 40, 1400, 64, 40)])
def test_decode_batch_roundtrip_and_oracle(sh, k, m, B, G, e_fixed):
    """BASELINE configs[2] (8192 x k=200 m=32 1400B, random erasures up to 32): every group's
    recovered blocks equal the erased originals (encode -> erase -> decode round trip, whole
    batch), the row rewrite follows the reference contract, and sampled groups match the oracle
    byte for byte."""
    import torch
    cfg = 0xD3 + k
    data, rec, blocks, d_rows, rows, es = _decode_inputs(k, m, B, G, cfg, e_fixed)
    orig_blocks = blocks.clone()
    assert sh.decode_batch(k, m, B, G, blocks, d_rows) == 0
    _sync()
    new_rows = d_rows.cpu().numpy()
    # rows: originals unchanged, recovery blocks -> erasures ascending in array order
    for g in range(0, G, max(1, G // 64)):
        present = set(int(r) for r in rows[g] if r < k)
        missing = [x for x in range(k) if x not in present]
        rec_pos = [i for i in range(k) if rows[g][i] >= k]
        exp = rows[g].copy()
        for i, p in enumerate(rec_pos):
            exp[p] = missing[i]
        assert np.array_equal(new_rows[g], exp), g
    # data: every block equals original data[row] (whole batch, on device)
    idx = torch.from_numpy(new_rows).cuda().long()
    truth = data[torch.arange(G, device="cuda")[:, None], idx]
    assert torch.equal(blocks, truth)
    # sampled groups vs the oracle's own decode
    ora = po.oracle()
    for g in sorted({0, G // 3, G - 1}):
        b = [x.copy() for x in orig_blocks[g].cpu().numpy()]
        rc, nr = ora.decode(k, m, b, list(rows[g]), B)
        assert rc == 0 and nr == new_rows[g].tolist()
        assert np.array_equal(np.stack(b), blocks[g].cpu().numpy())


# Off-grid (k, m): the runtime-coefficient tile kernels (csrc/tile_snip.hip) -- every part count
# (tile_parts: 1, 2, 4, 6, 8, 12, 16 parts of 4..8 rows; m = 3, 10, 24, 40, 60, 76, 100), two
# launches (m > 128), the shapes Shorthair's policy issues between the compiled pairs, and odd group
# counts (partial tiles).
TILE_SHAPES = [(120, 136, 1400, 37), (150, 44, 1400, 301), (50, 10, 1000, 513), (180, 76, 1352, 45),
               (2, 254, 128, 61), (100, 100, 200, 77), (5, 3, 128, 999), (70, 72, 520, 130),
               (17, 5, 1352, 9), (60, 24, 4104, 11), (33, 33, 136, 257), (240, 16, 264, 40),
               (150, 60, 1400, 33), (90, 49, 512, 70)]


@pytest.mark.parametrize("k,m,B,G", TILE_SHAPES)
def test_tile_encode_decode_vs_oracle(sh, k, m, B, G):
    """Encode and decode of shapes without compile-time kernels run on the tile kernels (path 2):
    encode bit-exact against the oracle on sampled groups; decode (random e up to min(k, m))
    recovers every group of the batch and matches the oracle's decode on sampled groups."""
    import torch
    assert sh.path(k, m, B) == "tile"
    cfg = 0x7E + k + m
    data, rec, blocks, d_rows, rows, es = _decode_inputs(k, m, B, G, cfg, 0)
    sample = sorted({0, G // 2, G - 1})
    exp = _oracle_encode_groups(k, m, B, cfg, sample)
    for g in sample:
        assert np.array_equal(rec[g].cpu().numpy(), exp[g][1]), f"encode g={g}"
    orig = blocks.clone()
    assert sh.decode_batch(k, m, B, G, blocks, d_rows) == 0
    _sync()
    new_rows = d_rows.cpu().numpy()
    truth = data[torch.arange(G, device="cuda")[:, None], torch.from_numpy(new_rows).cuda().long()]
    assert torch.equal(blocks, truth), "round trip"
    ora = po.oracle()
    for g in sample:
        b = [x.copy() for x in orig[g].cpu().numpy()]
        rc, nr = ora.decode(k, m, b, list(rows[g]), B)
        assert rc == 0 and nr == new_rows[g].tolist()
        assert np.array_equal(np.stack(b), blocks[g].cpu().numpy()), g


def test_decode_batch_out_matches_inplace(sh):
    import torch
    k, m, B, G = 200, 32, 1400, 512
    data, rec, blocks, d_rows, rows, es = _decode_inputs(k, m, B, G, 0xAB, 0)
    emax = min(k, m)
    out = torch.zeros((G, emax, B), dtype=torch.uint8, device="cuda")
    out_rows = torch.zeros((G, emax), dtype=torch.uint8, device="cuda")
    out_cnt = torch.zeros(G, dtype=torch.int32, device="cuda")
    assert sh.decode_batch_out(k, m, B, G, blocks, d_rows, out, out_rows, out_cnt) == 0
    _sync()
    cnt = out_cnt.cpu().numpy()
    assert np.array_equal(cnt, es)
    orow = out_rows.cpu().numpy()
    for g in range(G):
        e = int(cnt[g])
        truth = data[g, torch.from_numpy(orow[g, :e]).long().cuda()]
        assert torch.equal(out[g, :e], truth), g


def test_decode_no_erasures_and_invalid(sh):
    """Groups with nothing erased are untouched; invalid parameters return -1 only when some
    group has something to recover (reference cauchy_256.cpp:1266-1273)."""
    import torch
    k, m, B, G = 20, 4, 64, 5
    blocks = torch.randint(0, 256, (G, k, B), dtype=torch.uint8, device="cuda")
    rows = torch.arange(k, dtype=torch.uint8, device="cuda").repeat(G, 1).contiguous()
    before = blocks.clone()
    assert sh.decode_batch(k, m, B, G, blocks, rows) == 0
    _sync()
    assert torch.equal(blocks, before)
    assert sh.decode_batch(k, m, 12, G, blocks, rows) == 0  # B % 8 != 0 but nothing to do
    rows2 = rows.clone()
    rows2[1, 3] = k + 1
    assert sh.decode_batch(k, m, 12, G, blocks, rows2) == -1
    assert sh.decode_batch(200, 60, 16, 1, torch.zeros((1, 200, 16), dtype=torch.uint8, device="cuda"),
                           torch.full((1, 200), 200, dtype=torch.uint8, device="cuda")) == -1


def test_tiny_and_odd_block_sizes(sh):
    """B = 8/16/24 (sub-blocks shorter than a word) and B % 32 != 0 tails, encode + decode."""
    ora = po.oracle()
    rng = np.random.default_rng(7)
    import torch
    for B in (8, 16, 24, 40, 56, 1352, 1336, 1344, 4104):
        k, m = 17, 5
        G = 9
        data = rng.integers(0, 256, (G, k, B), dtype=np.uint8)
        d_out = torch.zeros((G, m, B), dtype=torch.uint8, device="cuda")
        assert sh.encode_batch(k, m, B, G, _dev(data), d_out) == 0
        _sync()
        for g in range(G):
            _, exp = ora.encode(k, m, data[g], B)
            assert np.array_equal(d_out[g].cpu().numpy(), exp), (B, g)


def test_decode_two_streams_concurrent(sh):
    """Two batched decodes in flight at once on two streams, different erasure patterns: each
    stream has its own decode workspace, so both results are exact."""
    import torch
    k, m, B, G = 200, 32, 1400, 768
    runs = []
    for cfg in (0x11, 0x22):
        data, rec, blocks, d_rows, rows, es = _decode_inputs(k, m, B, G, cfg, 0)
        out = torch.zeros((G, m, B), dtype=torch.uint8, device="cuda")
        orow = torch.zeros((G, m), dtype=torch.uint8, device="cuda")
        ocnt = torch.zeros(G, dtype=torch.int32, device="cuda")
        runs.append((data, blocks, d_rows, es, out, orow, ocnt, torch.cuda.Stream()))
    _sync()
    for _ in range(3):
        for data, blocks, d_rows, es, out, orow, ocnt, st in runs:
            with torch.cuda.stream(st):
                assert sh.decode_batch_out(k, m, B, G, blocks, d_rows, out, orow, ocnt,
                                           stream=st.cuda_stream) == 0
    _sync()
    for data, blocks, d_rows, es, out, orow, ocnt, st in runs:
        assert np.array_equal(ocnt.cpu().numpy(), es)
        idx = orow.long()
        truth = data[torch.arange(G, device="cuda")[:, None], idx]
        mask = torch.arange(m, device="cuda")[None, :] < ocnt[:, None]
        assert torch.equal(out[mask], truth[mask])


@pytest.mark.parametrize("k,m,B", [(28, 4, 256), (28, 4, 1400), (20, 6, 1400), (40, 2, 512),
                                   (250, 6, 1400), (33, 3, 256)])
def test_searched_table_setup_mixed_groups(sh, k, m, B):
    """m <= 6 setup (decode_setup_small: eight groups per wave, eight lanes per group) with every
    kind of group side by side in one wave: random e = 1..m in random array order, nothing erased
    (e = 0), a recovery row listed twice, a row past the generator. Counts, recovered blocks and
    rows against the oracle; the malformed groups are counted and left untouched."""
    import torch
    ora = po.oracle()
    rng = np.random.default_rng(k * 31 + m * 7 + B)
    G = 77
    data = rng.integers(0, 256, (G, k, B), dtype=np.uint8)
    rows = np.zeros((G, k), np.uint8)
    blocks = np.zeros((G, k, B), np.uint8)
    exp_cnt = np.zeros(G, np.int64)
    for g in range(G):
        rc, rec = ora.encode(k, m, data[g], B)
        assert rc == 0
        whole = np.concatenate([data[g], rec])
        kind = g % 7
        e = 0 if kind == 3 else int(rng.integers(1, min(k, m) + 1))
        lost = rng.choice(k, size=e, replace=False)
        recv = k + rng.choice(m, size=e, replace=False)
        r = np.array(sorted(set(range(k)) - set(lost.tolist())) + recv.tolist())
        rng.shuffle(r)
        if kind == 5 and e >= 1:       # a recovery row listed twice
            i0 = int(np.flatnonzero(r >= k)[0])
            j0 = int(np.flatnonzero(r < k)[0])
            r[j0] = r[i0]
        elif kind == 6 and k + m < 256:  # a row past the generator (a byte value)
            r[int(rng.integers(k))] = k + m
        rows[g] = r
        blocks[g] = whole[np.minimum(r, k + m - 1)]  # a malformed group's bytes are never read
        exp_cnt[g] = -1 if (kind == 5 and e >= 1) or (kind == 6 and k + m < 256) else e
    d_blocks, d_rows = _dev(blocks), _dev(rows)
    out = torch.zeros((G, m, B), dtype=torch.uint8, device="cuda")
    orow = torch.zeros((G, m), dtype=torch.uint8, device="cuda")
    ocnt = torch.zeros(G, dtype=torch.int32, device="cuda")
    sh.batch_errors()
    assert sh.decode_batch_out(k, m, B, G, d_blocks, d_rows, out, orow, ocnt) == 0
    assert sh.batch_errors() == int((exp_cnt < 0).sum())
    cnt = ocnt.cpu().numpy()
    assert np.array_equal(cnt, exp_cnt)
    o, orr = out.cpu().numpy(), orow.cpu().numpy()
    for g in range(G):
        e = int(cnt[g])
        if e <= 0:
            continue
        b = [x.copy() for x in blocks[g]]
        rc, nr = ora.decode(k, m, b, rows[g].tolist(), B)
        assert rc == 0
        rec_pos = [i for i in range(k) if rows[g][i] >= k]
        assert [nr[p] for p in rec_pos] == orr[g, :e].tolist(), g
        for l, p in enumerate(rec_pos):
            assert np.array_equal(o[g, l], b[p]), (g, l)
            assert np.array_equal(o[g, l], data[g, nr[p]]), (g, l)
    # in-place form: valid groups decoded, malformed ones untouched
    d_rows2 = _dev(rows)
    assert sh.decode_batch(k, m, B, G, d_blocks, d_rows2) == 0
    assert sh.batch_errors() == int((exp_cnt < 0).sum())
    nb, nr2 = d_blocks.cpu().numpy(), d_rows2.cpu().numpy()
    for g in range(G):
        if exp_cnt[g] < 0:
            assert np.array_equal(nb[g], blocks[g]) and np.array_equal(nr2[g], rows[g]), g
        else:
            assert np.array_equal(nb[g], data[g, nr2[g].astype(np.int64)]), g


@pytest.mark.parametrize("k,m,B", [(50, 10, 1000), (8, 20, 1400), (64, 16, 264), (12, 7, 1400),
                                   (40, 12, 256), (241, 15, 256), (100, 16, 256), (28, 4, 256),
                                   (20, 6, 1400), (20, 4, 1400), (250, 6, 1400), (40, 2, 512)])
def test_multi_group_setup_mixed_groups_many(sh, k, m, B):
    """More than 8192 groups, where the multi-group setups run (m >= 7 with emax <= 16:
    decode_setup_cauchy, 16 lanes per group; m <= 6: decode_setup_small, 8 lanes per group):
    random e and array order, e = 0, duplicated and out-of-range rows side by side. Counts and
    error count exact, every valid group's recovered blocks equal the encoded originals, row
    contract and bytes of sampled groups against the oracle's decode."""
    import torch
    G = 8300
    rng = np.random.default_rng(k * 131 + m)
    data = torch.empty((G, k, B), dtype=torch.uint8, device="cuda")
    rec = torch.empty((G, m, B), dtype=torch.uint8, device="cuda")
    assert sh.fill_synthetic(data, k, B, G, 0, 0x3C) == 0
    assert sh.encode_batch(k, m, B, G, data, rec) == 0
    emax = min(k, m)
    rows = np.zeros((G, k), np.int64)
    exp_cnt = np.zeros(G, np.int64)
    for g in range(G):
        kind = g % 7
        e = 0 if kind == 3 else int(rng.integers(1, emax + 1))
        lost = rng.choice(k, size=e, replace=False)
        recv = k + rng.choice(m, size=e, replace=False)
        keep = np.setdiff1d(np.arange(k), lost)
        r = np.concatenate([keep, recv])
        rng.shuffle(r)
        if kind == 5 and e >= 1:      # a recovery row listed twice (over an original if any)
            i0 = int(np.flatnonzero(r >= k)[0])
            others = np.flatnonzero(np.arange(k) != i0)
            r[int(others[0])] = r[i0]
        elif kind == 6 and k + m < 256:  # a row past the generator (a byte value)
            r[int(rng.integers(k))] = k + m
        rows[g] = r
        exp_cnt[g] = -1 if (kind == 5 and e >= 1) or (kind == 6 and k + m < 256) else e
    whole = torch.cat([data, rec], dim=1)
    d_rows = torch.from_numpy(rows.astype(np.uint8)).cuda()
    idx = torch.from_numpy(np.minimum(rows, k + m - 1)).cuda()
    blocks = whole[torch.arange(G, device="cuda")[:, None], idx].contiguous()
    del whole
    out = torch.zeros((G, emax, B), dtype=torch.uint8, device="cuda")
    orow = torch.zeros((G, emax), dtype=torch.uint8, device="cuda")
    ocnt = torch.zeros(G, dtype=torch.int32, device="cuda")
    sh.batch_errors()
    assert sh.decode_batch_out(k, m, B, G, blocks, d_rows, out, orow, ocnt) == 0
    assert sh.batch_errors() == int((exp_cnt < 0).sum())
    cnt = ocnt.cpu().numpy()
    assert np.array_equal(cnt, exp_cnt)
    # recovered blocks = the originals named by out_rows (valid groups, first e entries)
    valid = torch.from_numpy(cnt).cuda()
    truth = data[torch.arange(G, device="cuda")[:, None], orow.long()]
    mask = torch.arange(emax, device="cuda")[None, :] < valid[:, None]
    assert torch.equal(out[mask], truth[mask])
    # out_rows: the erased originals ascending (reference row contract)
    orr = orow.cpu().numpy()
    for g in range(0, G, 97):
        e = int(cnt[g])
        if e > 0:
            missing = np.setdiff1d(np.arange(k), rows[g][rows[g] < k])[:e]
            assert orr[g, :e].tolist() == missing.tolist(), g
    ora = po.oracle()
    for g in (1, G // 2 + 1, G - 2):
        if exp_cnt[g] <= 0:
            continue
        b = [x.copy() for x in blocks[g].cpu().numpy()]
        rc, nr = ora.decode(k, m, b, rows[g].tolist(), B)
        assert rc == 0
        rec_pos = [i for i in range(k) if rows[g][i] >= k]
        o = out[g].cpu().numpy()
        for l, p in enumerate(rec_pos):
            assert nr[p] == orr[g, l] and np.array_equal(o[l], b[p]), (g, l)


def test_malformed_groups_reported(sh):
    """A row listed twice (outside the reference's contract) leaves the group untouched, flags it
    with count -1 and is counted by cauchy_256_batch_errors; the single-group call returns -1."""
    import torch
    k, m, B, G = 40, 8, 64, 4
    assert sh.batch_errors() == 0
    blocks = torch.randint(0, 256, (G, k, B), dtype=torch.uint8, device="cuda")
    rows = torch.arange(k, dtype=torch.uint8, device="cuda").repeat(G, 1).contiguous()
    rows[:, 0] = k       # every group: original 0 lost, recovery row 0 received (valid)
    rows[2, 1] = k       # group 2: recovery row 0 listed twice (malformed)
    before = blocks.clone()
    out = torch.zeros((G, m, B), dtype=torch.uint8, device="cuda")
    orow = torch.zeros((G, m), dtype=torch.uint8, device="cuda")
    ocnt = torch.zeros(G, dtype=torch.int32, device="cuda")
    assert sh.decode_batch_out(k, m, B, G, blocks, rows, out, orow, ocnt) == 0
    assert sh.batch_errors() == 1
    assert ocnt.cpu().numpy().tolist() == [1, 1, -1, 1]
    r2 = rows.clone()
    assert sh.decode_batch(k, m, B, G, blocks, r2) == 0
    assert sh.batch_errors() == 1
    assert torch.equal(blocks[2], before[2]) and torch.equal(r2[2], rows[2])
    bufs = [np.zeros(B, np.uint8) for _ in range(k)]
    arr = (sh.Block * k)()
    rr = rows[2].cpu().numpy()
    for i in range(k):
        arr[i].data = bufs[i].ctypes.data
        arr[i].row = int(rr[i])
    assert sh.cauchy_256_decode(k, m, arr, B) == -1
    # counts are per stream: the single-group ABI decodes on private staging streams and reports
    # through its return code only, so no batch stream's count moves
    assert sh.batch_errors() == 0
    assert sh.batch_errors(sh.default_stream()) == 0


def test_c5_per_gpu_shard_131072_groups(sh):
    """BASELINE config C5 at its per-GPU shard size (1M groups over 8 GPUs = 131,072 groups of
    k=200 m=32 B=1400 per GPU, 36.7 GB of input): one encode and one in-place decode launch over
    the whole shard (every per-workgroup descriptor / 64-bit offset path at that size), the
    encode -> erase -> decode round trip checked for EVERY group on the device, and sampled
    groups (first, middle, last) against the oracle byte for byte."""
    import torch
    k, m, B, G, cfg = 200, 32, 1400, 131072, 0xC5
    data = torch.empty((G, k, B), dtype=torch.uint8, device="cuda")
    rec = torch.empty((G, m, B), dtype=torch.uint8, device="cuda")
    assert sh.fill_synthetic(data, k, B, G, 0, cfg) == 0
    assert sh.encode_batch(k, m, B, G, data, rec) == 0
    rows = np.zeros((G, k), np.uint8)
    for g in range(G):
        rows[g] = sh.erasure_pattern(g, k, m, cfg, 0)[1]
    d_rows = torch.from_numpy(rows).cuda()
    gi = torch.arange(G, device="cuda")[:, None]
    whole = torch.cat([data, rec], dim=1)
    blocks = whole[gi, d_rows.long()]  # device memory peak ~ 4 x 37 GB of the 288 GB
    del whole
    sample = (0, G // 2, G - 1)
    recv = {g: blocks[g].cpu().numpy() for g in sample}
    assert sh.decode_batch(k, m, B, G, blocks, d_rows) == 0
    _sync()
    assert sh.batch_errors() == 0
    new_rows = d_rows.long()
    assert torch.equal(blocks, data[gi, new_rows]), "round trip"
    ora = po.oracle()
    for g in sample:
        d = po.fill_group(g, k, B, cfg)
        rc, exp = ora.encode(k, m, d, B)
        assert rc == 0 and np.array_equal(rec[g].cpu().numpy(), exp), g
        b = [x.copy() for x in recv[g]]
        rc, nr = ora.decode(k, m, b, list(rows[g]), B)
        assert rc == 0 and nr == d_rows[g].cpu().numpy().tolist(), g
        assert np.array_equal(np.stack(b), blocks[g].cpu().numpy()), g


def test_exported_field_tables_match_oracle(sh):
    """GFC256_MUL_TABLE / GFC256_DIV_TABLE (cauchy_256.cpp:346-386): after init, entry (y << 8) + x
    is x * y and x / y, the oracle's field (both full 64K tables)."""
    lib = sh.lib
    ora = po.oracle().lib
    mul = np.ctypeslib.as_array(ctypes.cast(ctypes.c_void_p.in_dll(lib, "GFC256_MUL_TABLE").value,
                                            ctypes.POINTER(ctypes.c_ubyte)), shape=(256, 256)).copy()
    div = np.ctypeslib.as_array(ctypes.cast(ctypes.c_void_p.in_dll(lib, "GFC256_DIV_TABLE").value,
                                            ctypes.POINTER(ctypes.c_ubyte)), shape=(256, 256)).copy()
    exp_mul = np.array([[ora.ora_gf_mul(x, y) for x in range(256)] for y in range(256)], np.uint8)
    exp_div = np.array([[ora.ora_gf_div(x, y) if y else 0 for x in range(256)] for y in range(256)], np.uint8)
    assert np.array_equal(mul, exp_mul)
    assert np.array_equal(div, exp_div)
    assert mul[0x80, 2] == 0x87  # 2 * 0x80 reduced by the polynomial 0x187
    ref = po.reference()  # the reference's own tables, when oracle/_ref was built
    if ref is not None:
        for name, ours in (("GFC256_MUL_TABLE", mul), ("GFC256_DIV_TABLE", div)):
            p = ctypes.c_void_p.in_dll(ref.lib, name).value
            theirs = np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_ubyte)), shape=(256, 256))
            assert np.array_equal(ours, theirs), name
