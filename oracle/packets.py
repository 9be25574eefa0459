"""CPU restatement of the reference protocol layer's codec framing -- TEST INFRASTRUCTURE ONLY.

Restates, one group at a time on the C oracle codec (pyoracle.oracle()):
  tx_group   Encoder::EncodeQueued (Shorthair.cpp:480-576) + GenerateRecoveryBlock (:580-609)
  rx_group   RecoverGroup (:704-761) over the packets OnData (:764-902) keeps for a group
Only tests/ import this module (the product, shorthair_amd, never does). The codec bytes are
pinned by tests/golden (the compiled reference); the framing is pinned by the cited lines, as the
reference's protocol layer does not compile unmodified.
"""
import numpy as np


def roundup8(x):
    return (x + 7) & ~7


def tx_group(codec, m, packets):
    """Recovery packets (bytes) for one group: None when EncodeQueued encodes nothing."""
    k = len(packets)
    if m < 1 or k <= 0 or k >= 256:  # :486-496
        return None
    if k + m > 256:  # :501-504
        m = 256 - k
    if k == 1:  # :507-523 and GenerateRecoveryBlock :587-596
        return [bytes([1, 0]) + bytes(packets[0])] * m
    largest = max(len(p) for p in packets)
    B = roundup8(2 + largest)  # :528-534
    blocks = np.zeros((k, B), np.uint8)
    for x, p in enumerate(packets):  # :540-557: [len u16 LE][payload][zeros]
        blocks[x, 0] = len(p) & 0xFF
        blocks[x, 1] = len(p) >> 8
        blocks[x, 2:2 + len(p)] = np.frombuffer(bytes(p), np.uint8)
    rc, rec = codec.encode(k, m, [blocks[x] for x in range(k)], B)
    assert rc == 0
    # :598-608: [k+i][k-1][m-1][block i]
    return [bytes([k + y, k - 1, m - 1]) + rec[y].tobytes() for y in range(m)]


def rx_group(codec, originals, recovery):
    """Packets RecoverGroup delivers for one group, as [(id, payload)], or None when the group
    is not decoded (OnData's CanRecover() false, all originals seen, or no recovery packet).
    originals: [(id, payload)] and recovery: [packet] in arrival order."""
    if not recovery:
        return None
    k = recovery[0][1] + 1
    if k == 1:  # :858-866
        return [(0, bytes(recovery[0][2:]))] if not originals else None
    if len(originals) >= k or len(originals) + len(recovery) < k:
        return None
    last = recovery[-1]
    m = last[2] + 1  # :878
    B = len(last) - 3  # :877
    datas, rows = [], []
    for oid, p in originals:  # :710-725
        b = np.zeros(B, np.uint8)
        b[0] = len(p) & 0xFF
        b[1] = len(p) >> 8
        b[2:2 + len(p)] = np.frombuffer(bytes(p), np.uint8)
        datas.append(b)
        rows.append(oid)
    for r in recovery[:k - len(originals)]:  # :727-735
        datas.append(np.frombuffer(bytes(r[3:]), np.uint8).copy())
        rows.append(r[0])
    rc, new_rows = codec.decode(k, m, datas, rows, B)
    assert rc == 0
    out = []
    missing = sorted(set(range(k)) - {o[0] for o in originals})
    for ii in range(len(originals), k):  # :741-756
        src = datas[ii]
        ln = int(src[0]) | (int(src[1]) << 8)
        if ln <= B - 2:
            # the i-th recovery block carries the i-th smallest missing id (cauchy_256.cpp:548-553);
            # m == 1 leaves its row >= k, so the id comes from the erasure list
            pid = new_rows[ii] if new_rows[ii] < k else missing[ii - len(originals)]
            out.append((pid, src[2:2 + ln].tobytes()))
    return out
