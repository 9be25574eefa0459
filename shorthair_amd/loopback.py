"""Deterministic fake-clock loopback over the batched packet-group API.

Restates catid/shorthair's tests/Tester.cpp ZeroLossTest (:224-240) with a counter instead of
its wall clock (``sleep_for(TICK_RATE)`` in a ``for (;;)``), so a run is a pure function of its
arguments and can be checked exactly:

* ZeroLossServer::Tick (:133-163): PKTS_PER_TICK = 10 payloads per tick, each
  ``[id u32 LE][len u32 LE][PCG(id) bytes]`` with ``len = 8 + Next() % 1343`` from the shared
  PCG (seeded 0, :225-226).
* ZeroLossServer::SendData (:100-115): every datagram (original or recovery packet) is dropped
  when the shared PCG's next draw is below ``0xffffffff * 0.1``.
* ZeroLossClient::OnPacket (:169-187): every delivered payload is checked against PCG(id).
* ShorthairCodec::Tick (Shorthair.cpp:1061-1188): every max_delay = 100 ms (20 ticks of 5 ms)
  the queued originals become one code group of N = k packets and R recovery packets:
  ``CalculateApproximate(plr, N, 0.001)`` where N*plr and N*(1-plr) are >= 10, else N*3*plr;
  for N >= 3 clamped to 1.5N + 1 above an overhead of 0.5 and raised to N*(1 + 0.2) below
  min_fec_overhead = 0.2 (:1149-1165), at least 2; EncodeQueued truncates m to 256 - k (:502-504).
  That is how the Tester's captured shapes arise (k = 200 → R = 240 → m = 56).

Differences from the reference, all outside the codec: the loss estimate is the configured
channel loss (the reference learns it from exchanged statistics), recovery packets go out at
the swap instead of being spread over the next interval, and ``batch`` consecutive code groups
are encoded in one ``shorthair_encode_groups`` call and every recoverable group of them decoded in
one ``shorthair_recover_groups`` call (the reference: one group per call, on one thread).

The codec calls go through ``shorthair_amd.groups`` (the GPU library); a test can pass another
object with the same two functions to check this driver itself.
"""
import math
import struct

import numpy as np

TICK_MS = 5           # Tester.cpp:18 TICK_RATE
PKTS_PER_TICK = 10    # Tester.cpp:19
MAX_SIZE = 1350       # Tester.cpp:136
MIN_SIZE = 8          # Tester.cpp:137
MAX_DELAY_MS = 100    # Tester.cpp:124 settings.max_delay
MIN_FEC_OVERHEAD = 0.2
M64 = (1 << 64) - 1
MUL = 6364136223846793005


class PCG:
    """SiameseTools.h:80-102 PCGRandom (Seed(y, x): stream y, state offset x)."""

    def __init__(self, y, x=0):
        self.state, self.inc = 0, ((y << 1) | 1) & M64
        self.next()
        self.state = (self.state + x) & M64
        self.next()

    def next(self):
        old = self.state
        self.state = (old * MUL + self.inc) & M64
        xs = (((old >> 18) ^ old) >> 27) & 0xFFFFFFFF
        rot = old >> 59
        return ((xs >> rot) | (xs << ((-rot) & 31))) & 0xFFFFFFFF


def pcg_bytes(ids, n):
    """Low bytes of the first n draws of PCG(id) for every id (vectorized across ids)."""
    ids = np.asarray(ids, dtype=np.uint64)
    with np.errstate(over="ignore"):
        inc = (ids << np.uint64(1)) | np.uint64(1)
        st = np.zeros_like(ids)
        mul = np.uint64(MUL)
        st = st * mul + inc            # Seed: Next() from state 0, x = 0, Next()
        st = st * mul + inc
        out = np.empty((len(ids), n), dtype=np.uint8)
        for j in range(n):
            old = st
            st = old * mul + inc
            xs = (((old >> np.uint64(18)) ^ old) >> np.uint64(27)) & np.uint64(0xFFFFFFFF)
            rot = old >> np.uint64(59)
            v = (xs >> rot) | (xs << ((np.uint64(32) - rot) & np.uint64(31)))
            out[:, j] = (v & np.uint64(0xFF)).astype(np.uint8)
    return out


def payload(pid, length, body=None):
    """Tester's datagram for id pid: [id u32][len u32][PCG(id) bytes 8..len)."""
    if body is None:
        body = pcg_bytes([pid], max(0, length - 8))[0]
    return struct.pack("<II", pid, length) + bytes(body[:max(0, length - 8)])


def _normal_q(n, r, p):  # Shorthair.cpp:257-265 NormalApproximation
    m = n + r
    u = m * p
    s = math.sqrt(u * (1.0 - p))
    return 0.5 * math.erfc(0.70710678118655 * (r - u - 0.5) / s)


def calculate_approximate(p, n, qtarget):  # Shorthair.cpp:270-309
    if n <= 0:
        return 0
    r = 1
    while r < (1 << 32):
        if _normal_q(n, r, p) < qtarget:
            break
        r <<= 1
    if _normal_q(n, r - 1, p) < qtarget:
        s = r >> 1
        r -= 1
        while s > 0:
            t = r ^ s
            if _normal_q(n, t, p) < qtarget:
                r = t
            s >>= 1
    return r + 1  # :304, taken on both paths


def recovery_count(n, plr):
    """ShorthairCodec::Tick's R for a swap with N queued packets (Shorthair.cpp:1130-1170)."""
    if n * plr >= 10.0 and n * (1 - plr) >= 10.0:
        r = calculate_approximate(plr, n, 0.001)
    else:
        r = int(n * 3 * plr)
    if n >= 3:
        rate = r / float(n)
        if rate > 0.5:
            r = int(n * 1.5) + 1
        elif rate < MIN_FEC_OVERHEAD:
            r = int(n * (1.0 + MIN_FEC_OVERHEAD))
        r = max(r, 2)
    else:
        r = 2
    return r


class Stats:
    def __init__(self):
        self.sent = self.direct = self.recovered = self.groups = self.decoded = 0
        self.rec_sent = self.rec_received = 0
        self.expected_recovered = 0   # missing originals of decodable groups (driver's own count)
        self.lost = 0                 # missing originals of groups that cannot be decoded
        self.uncoded = 0              # originals still queued when the run ends (never coded)
        self.shapes = {}              # (k, m, block_bytes) -> groups
        self.bad = []                 # (id, reason) of any delivery that failed a check

    @property
    def received(self):
        return self.direct + self.recovered

    def line(self):  # ZeroLossClient::Tick's report (Tester.cpp:218)
        return f"{self.received} of {self.sent} : {self.received / max(1, self.sent):.6f}"


def run(ticks, loss=0.1, seed=0, batch=8, codec=None, verify=True, plr=0.03, jitter_us=500):
    """Run the loopback for `ticks` ticks of the fake clock. Returns Stats.

    loss: channel drop rate (Tester's ENABLE_PACKETLOSS); plr: the loss estimate the sender's
    redundancy acts on (the reference's estimator starts at its floor, 0.03, and only moves once
    statistics are exchanged, which this loopback does not model); jitter_us: each tick lasts
    5 ms plus a deterministic 0..jitter_us from a separate PCG stream, so swaps fall after 19 or
    20 ticks and code groups have the Tester's k = 190 / 200 (0 = exact 5 ms ticks, k = 200).

    Every original is either delivered on arrival or, if its group can be decoded (originals +
    recovery packets received >= k), delivered by the decoder; the rest are lost. `verify`
    checks every delivered payload against PCG(id)."""
    if codec is None:
        from . import groups as codec
    prng = PCG(seed)
    clock_rng = PCG(seed, 0x7E57)
    thresh = int(0xFFFFFFFF * loss)
    st = Stats()
    next_id = 0
    now_us = last_swap_us = 0
    queue = []              # ids of the current code group (sender side)
    arrived = []            # per queued original: did it arrive?
    pending = []            # code groups waiting for the batched encode: (ids, payloads, arrived)
    payloads, lens = {}, {}

    def dropped():
        return prng.next() < thresh

    def flush():
        if not pending:
            return
        enc = codec.encode_groups([(min(recovery_count(len(p), plr), 256 - len(p)), p)
                                   for (_, p, _) in pending])
        rx = []
        for (ids, pk, got), rec in zip(pending, enc):
            st.groups += 1
            k = len(pk)
            bb = (2 + max(len(x) for x in pk) + 7) & ~7 if k > 1 else len(pk[0])
            key = (k, len(rec), bb)
            st.shapes[key] = st.shapes.get(key, 0) + 1
            st.rec_sent += len(rec)
            kept = [r for r in rec if not dropped()]  # SendData of each recovery packet
            st.rec_received += len(kept)
            orig = [(i, pk[i]) for i in range(k) if got[i]]
            missing = k - len(orig)
            if missing and len(orig) + len(kept) >= k:
                st.expected_recovered += missing
            else:
                st.lost += missing
            rx.append((orig, kept, ids))
        n, delivered = codec.recover_groups([(o, r) for (o, r, _) in rx])
        st.decoded += n
        for g, local, data in delivered:
            pid = rx[g][2][local]
            st.recovered += 1
            if verify and data != payloads[pid]:
                st.bad.append((pid, "recovered payload mismatch"))
        pending.clear()

    for _ in range(ticks):
        # client.Tick() then server.Tick() (Tester.cpp:237-238): the server sends this tick's
        # packets, then its codec ticks and swaps once max_delay has passed (Shorthair.cpp:1124)
        now_us += TICK_MS * 1000 + (clock_rng.next() % (jitter_us + 1) if jitter_us else 0)
        for _ in range(PKTS_PER_TICK):
            lens[next_id] = MIN_SIZE + prng.next() % (MAX_SIZE - MIN_SIZE + 1)
            got = not dropped()
            arrived.append(got)
            queue.append(next_id)
            next_id += 1
            st.sent += 1
            st.direct += got
        if (now_us - last_swap_us) // 1000 >= MAX_DELAY_MS and queue:
            last_swap_us = now_us
            # the group's payloads (PCG vectorized over the group's ids)
            body = pcg_bytes(queue, max(lens[i] for i in queue) - 8)
            for j, pid in enumerate(queue):
                payloads[pid] = payload(pid, lens[pid], body[j])
            pending.append((list(queue), [payloads[i] for i in queue], list(arrived)))
            queue.clear()
            arrived.clear()
            if len(pending) >= batch:
                flush()
    flush()
    st.uncoded = len(queue)
    st.lost += sum(1 for a in arrived if not a)
    if verify:  # direct deliveries are the sender's own bytes; check the generator itself once
        for pid in [i for i in range(min(next_id, 64)) if i in payloads]:
            p = payloads[pid]
            pid2, ln = struct.unpack_from("<II", p)
            if pid2 != pid or ln != len(p) or p[8:] != bytes(pcg_bytes([pid], ln - 8)[0]):
                st.bad.append((pid, "generator"))
        if st.recovered != st.expected_recovered:
            st.bad.append((-1, f"recovered {st.recovered} != decodable-missing {st.expected_recovered}"))
        if st.received + st.lost != st.sent:
            st.bad.append((-1, "accounting"))
    return st


def main(argv=None):
    import argparse
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--ticks", type=int, default=2000)
    ap.add_argument("--loss", type=float, default=0.1)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--jitter-us", type=int, default=500)
    a = ap.parse_args(argv)
    st = run(a.ticks, a.loss, a.seed, a.batch, jitter_us=a.jitter_us)
    print(st.line(), f"groups={st.groups} decoded={st.decoded} recovered={st.recovered} lost={st.lost} "
          f"uncoded={st.uncoded} shapes(k,m,B)={sorted(st.shapes.items())} bad={st.bad[:3]}")
    return 1 if st.bad else 0


if __name__ == "__main__":
    raise SystemExit(main())
