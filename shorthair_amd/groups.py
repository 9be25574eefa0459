"""Packet-group framing on the GPU codec (include/shorthair_groups.h): ctypes binding.

Mirrors the reference protocol layer's use of the codec (catid/shorthair Shorthair.cpp):
``encode_groups`` = Encoder::EncodeQueued (:480-576) + GenerateRecoveryBlock (:580-609) for many
groups; ``recover_groups`` = RecoverGroup (:704-761) over the packets OnData (:764-902) keeps, for
many groups. Payloads are ``bytes``; recovery packets come back in the reference's wire framing
``[id][k-1][m-1][block]`` (k == 1: ``[1][0][payload]``).
"""
import ctypes

from . import _check, lib

_c = ctypes
_u8p = _c.POINTER(_c.c_ubyte)


class TxGroup(_c.Structure):
    _fields_ = [("k", _c.c_int), ("m", _c.c_int), ("packets", _c.POINTER(_c.c_void_p)),
                ("lens", _c.POINTER(_c.c_ushort)), ("out", _c.c_void_p), ("out_capacity", _c.c_int),
                ("m_out", _c.c_int), ("out_stride", _c.c_int)]


class RxGroup(_c.Structure):
    _fields_ = [("n_orig", _c.c_int), ("orig_ids", _c.c_void_p), ("orig_data", _c.POINTER(_c.c_void_p)),
                ("orig_lens", _c.POINTER(_c.c_ushort)), ("n_rec", _c.c_int),
                ("rec_packets", _c.POINTER(_c.c_void_p)), ("rec_lens", _c.POINTER(_c.c_int))]


ON_PACKET = _c.CFUNCTYPE(None, _c.c_void_p, _c.c_int, _c.c_int, _u8p, _c.c_int)

lib.shorthair_recovery_packet_bytes.argtypes = [_c.c_int, _c.POINTER(_c.c_ushort)]
lib.shorthair_recovery_packet_bytes.restype = _c.c_int
lib.shorthair_encode_groups.argtypes = [_c.POINTER(TxGroup), _c.c_int]
lib.shorthair_encode_groups.restype = _c.c_int
lib.shorthair_recover_groups.argtypes = [_c.POINTER(RxGroup), _c.c_int, ON_PACKET, _c.c_void_p]
lib.shorthair_recover_groups.restype = _c.c_int


def _bufs(items):
    """Keep-alive ctypes buffers and a void* array over a list of bytes."""
    bufs = [_c.create_string_buffer(bytes(b), max(1, len(b))) for b in items]
    arr = (_c.c_void_p * max(1, len(bufs)))(*[_c.addressof(b) for b in bufs])
    return bufs, arr


def recovery_packet_bytes(k, lens):
    arr = (_c.c_ushort * max(1, k))(*lens)
    return lib.shorthair_recovery_packet_bytes(k, arr)


def encode_groups(groups):
    """groups: list of (m, [payload bytes, ...]). Returns, per group, the list of recovery packets
    (bytes) the reference sender would emit, or raises ValueError on invalid input (rc -1)."""
    keep, tx = [], (TxGroup * max(1, len(groups)))()
    outs = []
    for i, (m, packets) in enumerate(groups):
        k = len(packets)
        bufs, arr = _bufs(packets)
        lens = (_c.c_ushort * max(1, k))(*[len(p) for p in packets])
        stride = recovery_packet_bytes(k, [len(p) for p in packets]) if 1 <= k <= 255 else 0
        cap = max(1, stride) * max(0, min(m, 256 - k) if k < 256 else 0)
        out = _c.create_string_buffer(max(1, cap))
        keep += [bufs, arr, lens, out]
        outs.append(out)
        tx[i] = TxGroup(k, m, arr, lens, _c.addressof(out), cap, 0, 0)
    rc = _check(lib.shorthair_encode_groups(tx, len(groups)), "shorthair_encode_groups")
    if rc != 0:
        raise ValueError("shorthair_encode_groups: invalid arguments")
    res = []
    for i, out in enumerate(outs):
        raw = out.raw
        s = tx[i].out_stride
        res.append([raw[y * s:(y + 1) * s] for y in range(tx[i].m_out)])
    return res


def recover_groups(groups):
    """groups: list of (originals, recovery) with originals = [(id, payload bytes), ...] and
    recovery = [packet bytes, ...], both in arrival order. Returns (decoded_count, delivered) with
    delivered = [(group, id, payload bytes), ...] in delivery order."""
    keep, rx = [], (RxGroup * max(1, len(groups)))()
    for i, (orig, rec) in enumerate(groups):
        ids = (_c.c_ubyte * max(1, len(orig)))(*[o[0] for o in orig])
        obufs, oarr = _bufs([o[1] for o in orig])
        olens = (_c.c_ushort * max(1, len(orig)))(*[len(o[1]) for o in orig])
        rbufs, rarr = _bufs(rec)
        rlens = (_c.c_int * max(1, len(rec)))(*[len(r) for r in rec])
        keep += [ids, obufs, oarr, olens, rbufs, rarr, rlens]
        rx[i] = RxGroup(len(orig), _c.addressof(ids), oarr, olens, len(rec), rarr, rlens)
    delivered = []

    def on_packet(_ctx, group, pid, data, length):
        delivered.append((group, pid, _c.string_at(data, length)))

    cb = ON_PACKET(on_packet)
    rc = _check(lib.shorthair_recover_groups(rx, len(groups), cb, None), "shorthair_recover_groups")
    if rc < 0:
        raise ValueError("shorthair_recover_groups: malformed input")
    return rc, delivered
