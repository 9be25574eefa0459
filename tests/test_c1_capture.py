"""BASELINE config C1: real cauchy_256 calls of the reference's protocol layer, captured from
the reference's unchanged Shorthair.cpp running a Tester-shaped loopback on the reference codec
(tools/capture_c1.py, oracle/capture_wrap.cpp -> tests/golden/c1_capture.npz): Shorthair-framed
variable-length packets zero-padded to B = 1352 / 1344, k = 200 / 190, m = 256 - k, packet
pointers misaligned as the protocol leaves them. The oracle reproduces them on the CPU; the GPU
codec reproduces them through the single-group ABI with the captured pointer alignment and through
the batched API."""
import os

import numpy as np
import pytest

from oracle import pyoracle as po

ROOT = os.path.normpath(os.path.join(os.path.dirname(__file__), ".."))
Z = np.load(os.path.join(ROOT, "tests", "golden", "c1_capture.npz"))
ENC = sorted({f.split("_")[0] for f in Z.files if f.startswith("enc")})
DEC = sorted({f.split("_")[0] for f in Z.files if f.startswith("dec")})


def _kmb(p):
    k, m, B, rc = (int(x) for x in Z[p + "_kmbrc"])
    return k, m, B, rc


def _placed(blocks, align):
    """Host copies of the blocks at the captured address-mod-16 offsets: (buffer, offsets, ptrs)."""
    k, B = blocks.shape
    raw = np.zeros(k * (B + 32) + 64, np.uint8)
    base = (-raw.ctypes.data) % 16
    offs = [base + i * (B + 32) + int(align[i]) for i in range(k)]
    for i in range(k):
        raw[offs[i]:offs[i] + B] = blocks[i]
    return raw, offs, [raw.ctypes.data + o for o in offs]


def test_capture_shapes():
    assert ENC and DEC
    shapes = {_kmb(p)[:3] for p in ENC + DEC}
    assert (200, 56, 1352) in shapes and any(k == 190 and m == 66 for k, m, _ in shapes)
    assert any(int(a) % 4 for p in ENC for a in Z[p + "_align"]), "captured pointers are misaligned"


@pytest.mark.parametrize("p", ENC)
def test_oracle_reproduces_captured_encode(p):
    k, m, B, rc = _kmb(p)
    _, out = po.oracle().encode(k, m, Z[p + "_data"], B)
    assert rc == 0 and np.array_equal(out, Z[p + "_out"])


@pytest.mark.parametrize("p", DEC)
def test_oracle_reproduces_captured_decode(p):
    k, m, B, rc = _kmb(p)
    blocks = [x.copy() for x in Z[p + "_data_in"]]
    got_rc, rows = po.oracle().decode(k, m, blocks, list(Z[p + "_rows_in"]), B)
    assert got_rc == rc == 0 and rows == Z[p + "_rows_out"].tolist()
    idx = Z[p + "_idx"]
    assert np.array_equal(np.stack([blocks[i] for i in idx]), Z[p + "_data_out"])


@pytest.fixture(scope="module")
def sh():
    import torch
    import shorthair_amd
    assert shorthair_amd.cauchy_256_init() == 0
    torch.cuda.init()
    return shorthair_amd


@pytest.mark.gpu
@pytest.mark.parametrize("p", ENC)
def test_gpu_single_group_encode_captured(sh, p):
    k, m, B, rc = _kmb(p)
    raw, offs, ptrs = _placed(Z[p + "_data"], Z[p + "_align"])
    out = np.zeros(m * B + 16, np.uint8)
    assert sh.cauchy_256_encode(k, m, ptrs, out.ctypes.data + 3, B) == rc
    assert np.array_equal(out[3:3 + m * B].reshape(m, B), Z[p + "_out"])


@pytest.mark.gpu
@pytest.mark.parametrize("p", DEC)
def test_gpu_single_group_decode_captured(sh, p):
    k, m, B, rc = _kmb(p)
    raw, offs, ptrs = _placed(Z[p + "_data_in"], Z[p + "_align"])
    arr = (sh.Block * k)()
    rows_in = Z[p + "_rows_in"]
    for i in range(k):
        arr[i].data = ptrs[i]
        arr[i].row = int(rows_in[i])
    assert sh.cauchy_256_decode(k, m, arr, B) == rc
    assert [arr[i].row for i in range(k)] == Z[p + "_rows_out"].tolist()
    got = np.stack([raw[offs[i]:offs[i] + B] for i in Z[p + "_idx"]])
    assert np.array_equal(got, Z[p + "_data_out"])


@pytest.mark.gpu
@pytest.mark.parametrize("p", DEC)
def test_gpu_batch_decode_captured(sh, p):
    """The same calls as a batch of 3 copies through the device-resident API."""
    import torch
    k, m, B, rc = _kmb(p)
    G = 3
    blocks = torch.from_numpy(np.stack([Z[p + "_data_in"]] * G)).cuda()
    rows = torch.from_numpy(np.stack([Z[p + "_rows_in"]] * G)).cuda()
    assert sh.decode_batch(k, m, B, G, blocks, rows) == 0
    torch.cuda.synchronize()
    for g in range(G):
        assert rows[g].cpu().numpy().tolist() == Z[p + "_rows_out"].tolist()
        assert np.array_equal(blocks[g].cpu().numpy()[Z[p + "_idx"]], Z[p + "_data_out"])
