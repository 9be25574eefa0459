#!/usr/bin/env python3
"""Benchmark: batched cauchy_256 encode + decode, device-resident, on 1..8 MI355X GPUs.

One step = encode a batch of code groups (k data -> m recovery blocks each) + decode the same
number of groups with e erased originals each (read k received blocks, write e recovered ones),
inputs already resident in HBM. Headline config (BASELINE.json metric): k=200, m=32, 1400-byte
blocks, e = m = 32 (worst case), 8192 groups per GPU. Multi-GPU: one process per GPU, groups
sharded with no data-path collective (independent units -> weak scaling); timing is bracketed by
barrier + synchronize and the max over ranks is reported.

value = algorithmic GiB/s over all ranks: encode moves (k+m)*B and decode (k+e)*B bytes per group
(SURVEY.md §8d). roofline: the dominant kernel -- decode stage A, timed by the library's own HIP
events around that launch on its stream (cauchy_256_profile(-steps): the only events inside the
timed steps), or the encode kernel if that takes longer (timed in the breakdown pass); both move
(k+m)*B algorithmic bytes per group (read k blocks, write m rows) -- against the 8 TB/s HBM3E
peak. The per-op split (encode, decode, setup / stage A / stage B) is an equal second pass of
steps recorded with every event, after the timed steps: event packets between the kernels cost
~1.3 % of a step (profiles/r06/ab_runs.txt block 4) and are kept out of the headline.
cpu_baseline: the reference codec (oracle/_ref, compiled from catid/shorthair) on the host cores,
rank 0 only, bounded sample.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK = 8.0e12  # B/s, MI355X HBM3E spec (MI355X_MICROARCH.md chip table)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--settle-steps", type=int, default=40,
                   help="untimed steps before the warm-up: the GPU's power management needs ~20-30 "
                        "steps of sustained load after idle to settle its clock (tools/ramp_probe.py)")
    p.add_argument("--k", type=int, default=200)
    p.add_argument("--m", type=int, default=32)
    p.add_argument("--block", type=int, default=1400)
    p.add_argument("--groups", type=int, default=8192, help="code groups per GPU per op")
    p.add_argument("--total-groups", type=int, default=0,
                   help="code groups of the whole job per op, sharded over the ranks (C5: 1048576 over 8 "
                        "GPUs); overrides --groups")
    p.add_argument("--root-chunk", type=int, default=0,
                   help="N>1 root-resident leg: groups per rank per RCCL scatter/gather chunk (0 = as many as "
                        "fit a ~16 GB window on the root)")
    p.add_argument("--erasures", type=int, default=32, help="erasures per decoded group (0=random 1..m)")
    p.add_argument("--cpu-seconds", type=float, default=4.0, help="CPU baseline: seconds per mode")
    p.add_argument("--cpu-threads", type=int, default=0, help="0 = all host cores of this job")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--host-calls", type=int, default=50, help="single-group ABI calls timed (0 = skip)")
    p.add_argument("--host-groups", type=int, default=1024, help="groups of the pinned-host batch leg")
    p.add_argument("--root-steps", type=int, default=3,
                   help="N>1: steps of the root-resident variant (RCCL scatter -> encode -> gather); 0 = skip")
    p.add_argument("--no-sweep", action="store_true", help="skip the C2/C3/C4/Tester-shape leg")
    p.add_argument("--pg-timeout", type=int, default=120,
                   help="N>1: torch.distributed collective timeout in seconds (nccl backend)")
    p.add_argument("--backend", default="nccl",
                   help="torch.distributed backend for N > 1 (nccl = RCCL; gloo only to rehearse the "
                        "multi-rank path with several ranks on one GPU)")
    p.add_argument("--dry-run", action="store_true",
                   help="launcher check without a GPU: ranks join a gloo group and rank 0 reports them")
    return p.parse_args()


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch(args):
    """`--gpus N` outside a launcher: start N rank processes of this script (one per GPU, rank r on
    device r) with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set, and wait for
    them. The parent never touches the GPU (it does not even import torch); rank 0 prints the
    JSON line. Returns the first non-zero rank exit code."""
    import subprocess
    port = str(free_port())
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    return next((rc for rc in rcs if rc != 0), 0)


def dry_run(args, rank, world, local):
    """Launcher check (no GPU): every rank joins a gloo group over 127.0.0.1 and rank 0 prints
    what each rank saw."""
    import torch
    import torch.distributed as dist
    if world == 1:
        os.environ.update(RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()))
    dist.init_process_group("gloo")
    me = torch.tensor([rank, local, world, int(os.environ.get("MASTER_PORT", "0")), os.getpid()])
    allr = [torch.zeros_like(me) for _ in range(dist.get_world_size())]
    dist.all_gather(allr, me)
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": dist.get_world_size(), "gpus_arg": args.gpus,
                          "ranks": [dict(zip(("rank", "local_rank", "world_size", "master_port", "pid"),
                                             [int(v) for v in t])) for t in allr]}), flush=True)
    dist.destroy_process_group()


def host_cores():
    """CPUs this process may use (the GPU box gives each job a share of a large host: the
    affinity mask / OMP_NUM_THREADS, not os.cpu_count(), says how many)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(omp))) if omp and omp.isdigit() else n


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(k, m, B, e_fixed, seconds, threads):
    """The reference codec (oracle/_ref/libref_cauchy.so, compiled from catid/shorthair by
    oracle/Makefile) timed by the native pthreads harness oracle/_ref/cpu_bench on this host:
    1 thread and `threads` threads, as shipped (gf256_init not called) and after gf256_init()
    (AVX2 XOR helpers). Same synthetic inputs as the GPU run. `value` is the fastest mode at
    `threads` threads. Returns None when the harness is absent."""
    import subprocess
    exe = os.path.join(ROOT, "oracle", "_ref", "cpu_bench")
    if not os.path.exists(exe):
        return None
    modes = {}
    for t in sorted({1, threads}):
        for mode in ("shipped", "init"):
            r = subprocess.run([exe, str(k), str(m), str(B), str(e_fixed or m), str(t), str(seconds), mode],
                               capture_output=True, text=True, timeout=seconds * 4 + 60)
            if r.returncode != 0:
                return None
            kv = dict(x.split("=") for x in r.stdout.split())
            modes[f"{mode}_t{t}"] = {"GiBps": float(kv["GiBps"]), "groups": int(kv["groups"]),
                                     "us_per_encode": float(kv["us_per_encode"]),
                                     "us_per_decode": float(kv["us_per_decode"])}
    best = max((modes[f"{md}_t{threads}"]["GiBps"], md) for md in ("shipped", "init"))
    return dict(value=round(best[0], 4), unit="GiB/s", cores=threads, kind="reference",
                sample=f"native pthreads harness (oracle/cpu_bench.c), {seconds:g}s per mode, encode+decode "
                       f"group pairs k={k} m={m} B={B} e={e_fixed or m}, reference built -O3 -march=x86-64-v3; "
                       f"value = {best[1]} at {threads} threads",
                cpu=cpu_model(), modes=modes)


def root_resident(args, sh, shd, dist, torch, rank, world, G, k, m, B, s, enc_in, enc_out,
                  dec_in, rows, dec_out, dec_rows, dec_cnt, es):
    """Groups start and end on rank 0's GPU (north_star's root-resident flow), for
    both ops, streamed through a window on the root (shd.RootStream: chunk j+1's RCCL scatter
    and chunk j's RCCL gather overlap chunk j's kernels):
      encode: scatter k*B data bytes per group, encode, gather m*B recovery bytes;
      decode: scatter the k*B received blocks + the k-byte row array per group, decode_batch_out,
              gather the e*B recovered blocks + their rows + the count.
    The root holds one window per op (~16 GB), never the whole batch, so the leg runs at C5 scale
    (1M groups: 280 GB of input, more than one GPU's HBM). The window's inputs are copies of the
    root's own first chunk of groups; after the warm-up pass the root codes its whole window
    itself and checks every rank's slot of the last chunk against it. Reported beside the main
    line, never as `value`."""
    sizes = [shd.shard(args.total_groups, world, r)[1] for r in range(world)] if args.total_groups else [G] * world
    emax = min(k, m)
    window = float(os.environ.get("SH_ROOT_WINDOW_BYTES", "16e9"))  # smaller: tests only
    out = {}

    def leg(name, per_group, ins, outs, compute, make_win, check):
        # --root-chunk is clamped to the largest shard (the root's: shard() gives the first ranks
        # the extra group), so the root's window, built from its own first `chunk` groups, always
        # holds world * chunk rows
        chunk = min(args.root_chunk, max(sizes)) if args.root_chunk else shd.root_chunk_size(sizes, per_group, window)
        assert sizes[0] >= chunk, "the root's shard must cover one chunk"
        rs = shd.RootStream(sizes, chunk, ins, outs)
        win_in = win_out = None
        if rank == 0:
            win_in = make_win(chunk)
            win_out = [torch.zeros((world * chunk,) + tuple(t.shape[1:]), dtype=t.dtype, device="cuda") for t in outs]
        torch.cuda.synchronize()
        rs.run(compute, win_in, win_out)  # warm-up, and the pass the check reads
        torch.cuda.synchronize()
        ok = check(rs, chunk, win_in, win_out) if rank == 0 else None
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.root_steps):
            rs.run(compute, win_in, win_out)
        torch.cuda.synchronize()
        dist.barrier()
        t = shd.max_over_ranks(time.perf_counter() - t0, device="cuda")
        del win_in, win_out
        return {"chunk_groups_per_rank": chunk, "chunks": rs.nchunks,
                "root_window_GB": round(world * chunk * per_group / 1e9, 2),
                "ms_per_step": round(t / args.root_steps * 1e3, 4), "seconds": t, "roundtrip_ok": ok}

    # ---- encode ----
    def enc_compute(lo, n):
        assert sh.encode_batch(k, m, B, n, enc_in[lo:], enc_out[lo:], s) == 0

    def enc_win(chunk):
        return [enc_in[:chunk].repeat(world, 1, 1)]

    def enc_check(rs, chunk, win_in, win_out):
        exp = torch.empty_like(win_out[0])
        assert sh.encode_batch(k, m, B, world * chunk, win_in[0], exp, s) == 0
        torch.cuda.synchronize()
        return all(bool(torch.equal(win_out[0][a:a + n], exp[a:a + n])) for _, a, n in rs.slots() if n)

    r = leg("encode", (k + m) * B, [enc_in], [enc_out], enc_compute, enc_win, enc_check)
    out["encode"] = dict(r, GiBps=round(sum(sizes) * (k + m) * B * args.root_steps / r.pop("seconds") / 2**30, 3),
                         op="per chunk: RCCL scatter of data blocks, encode, RCCL gather of recovery blocks")

    # ---- decode ----
    def dec_compute(lo, n):
        assert sh.decode_batch_out(k, m, B, n, dec_in[lo:], rows[lo:], dec_out[lo:], dec_rows[lo:],
                                   dec_cnt[lo:], s) == 0

    def dec_win(chunk):
        return [dec_in[:chunk].repeat(world, 1, 1), rows[:chunk].repeat(world, 1)]

    def dec_check(rs, chunk, win_in, win_out):
        n_all = world * chunk
        exp = [torch.empty_like(w) for w in win_out]
        assert sh.decode_batch_out(k, m, B, n_all, win_in[0], win_in[1], *exp, s) == 0
        torch.cuda.synchronize()
        ok = True
        for _, a, n in rs.slots():
            if not n:
                continue
            cnt = exp[2][a:a + n]
            ok &= bool(torch.equal(win_out[2][a:a + n], cnt))
            ok &= bool(torch.equal(cnt.cpu(), torch.from_numpy(es[:chunk]).int().repeat(world)[a:a + n]))
            mask = torch.arange(emax, device="cuda")[None, :] < cnt[:, None]
            ok &= bool(torch.equal(win_out[1][a:a + n][mask], exp[1][a:a + n][mask]))
            ok &= bool(torch.equal(win_out[0][a:a + n][mask], exp[0][a:a + n][mask]))
        return ok

    per_dec = k * B + k + emax * B + emax + 4
    r = leg("decode", per_dec, [dec_in, rows], [dec_out, dec_rows, dec_cnt], dec_compute, dec_win, dec_check)
    # Algorithmic bytes of the groups actually decoded: every rank's slot of chunk j holds copies
    # of the root's first n_rj groups (the window), so their erasure counts are the root's
    # es[:n_rj], not the rank's own. Only the root reports.
    dec_all = 0
    if rank == 0:
        per = np.concatenate([[0], np.cumsum(k + es[:r["chunk_groups_per_rank"]].astype(np.int64))]) * B
        for j in range(r["chunks"]):
            for n in sizes:
                dec_all += int(per[max(0, min(r["chunk_groups_per_rank"], n - j * r["chunk_groups_per_rank"]))])
    out["decode"] = dict(r, GiBps=round(dec_all * args.root_steps / r.pop("seconds") / 2**30, 3),
                         op="per chunk: RCCL scatter of received blocks + rows, decode, RCCL gather of "
                            "recovered blocks + rows + counts")
    if rank != 0:
        return None
    out["steps"] = args.root_steps
    out["overlap"] = "chunk j+1 scatter and chunk j gather posted async around chunk j's kernels"
    out["roundtrip_ok"] = bool(out["encode"]["roundtrip_ok"] and out["decode"]["roundtrip_ok"])
    return out


def host_path(args, sh, torch, k, m, B, s):
    """PCIe-inclusive rates (never `value`): (1) the reference-shaped single-group ABI on host
    pointers (cauchy_256_encode / cauchy_256_decode: pinned staging, H2D, kernels, D2H per call);
    (2) a batch that starts and ends in pinned host memory: H2D of the data, encode, D2H of the
    recovery blocks, timed on the stream as one pipeline."""
    import ctypes
    out = {}
    rng = np.random.default_rng(7)
    data = rng.integers(0, 256, size=(k, B), dtype=np.uint8)
    rec = np.empty((m, B), np.uint8)
    ptrs = [data[x].ctypes.data for x in range(k)]
    n1 = args.host_calls
    assert sh.cauchy_256_encode(k, m, ptrs, rec.ctypes.data, B) == 0  # warm-up
    t0 = time.perf_counter()
    for _ in range(n1):
        sh.cauchy_256_encode(k, m, ptrs, rec.ctypes.data, B)
    t_enc = (time.perf_counter() - t0) / n1
    # decode: e = m lost originals, fresh block copies per call prepared outside the timed loop
    e = min(m, k)
    whole = np.concatenate([data, rec])
    rows = list(range(e, k)) + list(range(k, k + e))
    sets = []
    for _ in range(n1 + 1):
        bufs = [whole[r].copy() for r in rows]
        arr = (sh.Block * k)(*[sh.Block(b.ctypes.data, r) for b, r in zip(bufs, rows)])
        sets.append((bufs, arr))
    assert sh.cauchy_256_decode(k, m, sets[0][1], B) == 0  # warm-up (staging growth), as for encode
    sets = sets[1:]
    t0 = time.perf_counter()
    for bufs, arr in sets:
        sh.cauchy_256_decode(k, m, arr, B)
    t_dec = (time.perf_counter() - t0) / n1
    ok = all(np.array_equal(sets[-1][0][k - e + i], data[i]) for i in range(e))
    out["single_group"] = {"encode_us": round(t_enc * 1e6, 1), "decode_us": round(t_dec * 1e6, 1),
                           "GiBps": round(2 * (k + m) * B / (t_enc + t_dec) / 2**30, 4),
                           "calls": n1, "decode_ok": bool(ok)}
    out["pinned_batch_encode"] = pinned_batch(args, sh, torch, k, m, B)
    out["pinned_batch_encode_serial"] = pinned_batch(args, sh, torch, k, m, B, chunks=1)
    out["packet_groups"] = packet_groups(args, k, m, B)
    return out


def pinned_batch(args, sh, torch, k, m, B, chunks=8):
    """A batch that starts and ends in pinned host memory: H2D of the data, encode, D2H of the
    recovery blocks. chunks > 1 pipelines it over three streams (copy-in, codec, copy-out; PCIe is
    full duplex), so chunk i's encode and D2H run under chunk i+1's H2D; chunks = 1 is the
    serial form. Bound: the H2D of k*B bytes per group over PCIe (63 GB/s spec, Gen5 x16)."""
    G = args.host_groups
    h_in = torch.empty((G, k, B), dtype=torch.uint8, pin_memory=True)
    h_rec = torch.empty((G, m, B), dtype=torch.uint8, pin_memory=True)
    d_in = torch.empty((G, k, B), dtype=torch.uint8, device="cuda")
    d_rec = torch.empty((G, m, B), dtype=torch.uint8, device="cuda")
    sh.fill_synthetic(d_in, k, B, G, 0, 0xBE)
    torch.cuda.synchronize()
    h_in.copy_(d_in)
    ref = d_rec.clone()
    assert sh.encode_batch(k, m, B, G, d_in, ref) == 0
    d_in.zero_()
    torch.cuda.synchronize()
    s_in, s_enc, s_out = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    bounds = [(G * i // chunks, G * (i + 1) // chunks) for i in range(chunks)]
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = None
    for _ in range(4):  # first pass warms up
        torch.cuda.synchronize()
        ev0.record(s_in)
        s_enc.wait_event(ev0)
        s_out.wait_event(ev0)
        for a, b in bounds:
            with torch.cuda.stream(s_in):
                d_in[a:b].copy_(h_in[a:b], non_blocking=True)
                landed = torch.cuda.Event()
                landed.record(s_in)
            s_enc.wait_event(landed)
            assert sh.encode_batch(k, m, B, b - a, d_in[a:], d_rec[a:], s_enc.cuda_stream) == 0
            coded = torch.cuda.Event()
            coded.record(s_enc)
            s_out.wait_event(coded)
            with torch.cuda.stream(s_out):
                h_rec[a:b].copy_(d_rec[a:b], non_blocking=True)
        ev1.record(s_out)
        torch.cuda.synchronize()
        ms = ev0.elapsed_time(ev1)
        best = ms if best is None else min(best, ms)
    ok = bool(torch.equal(h_rec, ref.cpu()))
    return {"groups": G, "chunks": chunks, "ms": round(best, 3),
            "GiBps": round(G * (k + m) * B / (best * 1e-3) / 2**30, 2),
            "h2d_GBps": round(G * k * B / (best * 1e-3) / 1e9, 1), "ok": ok,
            "note": ("H2D / encode / D2H pipelined over three streams" if chunks > 1 else
                     "H2D data + encode + D2H recovery, serial on one stream")}


def packet_groups(args, k, m, B):
    """Host packets -> wire recovery packets and back through include/shorthair_groups.h:
    reference framing on host threads, pinned staging, PCIe, kernels, double-buffered chunks.
    Payloads of B-2 bytes (block = B); the receiver lost e = m originals per group."""
    import ctypes
    from shorthair_amd import groups as sg
    G = args.host_groups
    rng = np.random.default_rng(11)
    pay = rng.integers(0, 256, size=(G, k, B - 2), dtype=np.uint8)
    lens = (ctypes.c_ushort * k)(*([B - 2] * k))
    ptrs = [(ctypes.c_void_p * k)(*[pay[g, x].ctypes.data for x in range(k)]) for g in range(G)]
    stride = 3 + B
    rec = np.zeros((G, m, stride), np.uint8)
    tx = (sg.TxGroup * G)(*[sg.TxGroup(k, m, ptrs[g], lens, rec[g].ctypes.data, m * stride, 0, 0)
                            for g in range(G)])
    assert sg.lib.shorthair_encode_groups(tx, G) == 0  # warm-up (allocates staging)
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        assert sg.lib.shorthair_encode_groups(tx, G) == 0
    t_tx = (time.perf_counter() - t0) / reps
    e = min(m, k)
    ids = (ctypes.c_ubyte * (k - e))(*range(e, k))
    optr = [(ctypes.c_void_p * (k - e))(*[pay[g, x].ctypes.data for x in range(e, k)]) for g in range(G)]
    olens = (ctypes.c_ushort * (k - e))(*([B - 2] * (k - e)))
    rptr = [(ctypes.c_void_p * e)(*[rec[g, y].ctypes.data for y in range(e)]) for g in range(G)]
    rlens = (ctypes.c_int * e)(*([stride] * e))
    rx = (sg.RxGroup * G)(*[sg.RxGroup(k - e, ctypes.addressof(ids), optr[g], olens, e, rptr[g], rlens)
                            for g in range(G)])
    null_cb = ctypes.cast(None, sg.ON_PACKET)
    got = []
    def keep(_ctx, g, pid, d, n):
        if g < 2:
            got.append((g, pid, ctypes.string_at(d, n)))
    cb = sg.ON_PACKET(keep)
    assert sg.lib.shorthair_recover_groups(rx, G, cb, None) == G  # warm-up + spot check
    ok = all(bytes(pay[g, pid]) == p for g, pid, p in got) and len(got) == 2 * e
    t0 = time.perf_counter()
    for _ in range(reps):
        assert sg.lib.shorthair_recover_groups(rx, G, null_cb, None) == G
    t_rx = (time.perf_counter() - t0) / reps
    wire = G * (k + m) * B
    return {"groups": G, "encode_ms": round(t_tx * 1e3, 2), "recover_ms": round(t_rx * 1e3, 2),
            "encode_GiBps": round(wire / t_tx / 2**30, 2), "recover_GiBps": round(G * (k + e) * B / t_rx / 2**30, 2),
            "delivered_ok": bool(ok), "host_threads": os.environ.get("SH_HOST_THREADS", "hw"),
            "note": "host payloads -> framed blocks (host threads) -> pinned -> GPU -> wire packets; "
                    "recover: decode only (no delivery callback) in the timed loop"}


# BASELINE.json config 2 (C2), config 4 (C4 sweep: k+m in {32,128,256} x B in {256,1400,64KiB},
# m = (k+m)/8 as SURVEY §8d suggests) and the shapes catid/shorthair's Tester actually issues
# (Shorthair.cpp:502-504 clamps m to 256-k).
SWEEP = [("C2", 64, 16, 1400), ("C2 4096 groups", 64, 16, 1400, 4096)] + [("C4", k, m, B) for (k, m) in ((28, 4), (112, 16), (224, 32))
                                  for B in (256, 1400, 65536)] + \
        [("tester", 200, 56, 1352), ("tester", 190, 66, 1336), ("tester", 190, 66, 1344)] + \
        [("off-grid", 120, 136, 1400), ("off-grid", 150, 40, 1400), ("off-grid", 50, 10, 1000),
         ("off-grid", 180, 76, 1352)] + \
        [("k < K", 150, 32, 1400), ("k < K", 150, 56, 1352), ("k < K", 120, 66, 1336)]  # fixed_kernel_k


def sweep(args, sh, torch, s):
    """Per-shape device time of encode and decode (e = m worst case) with algorithmic GB/s and
    fraction of the HBM peak, ~1.5 GB of input per op unless the entry fixes its group count (C2 at
    BASELINE.json's 4096 groups); plus C3 (random e in 1..32)."""
    out = []
    for tag, k, m, B, *fixed in SWEEP:
        G = fixed[0] if fixed else max(8, int(1.5e9 // (k * B)))
        data = torch.empty((G, k, B), dtype=torch.uint8, device="cuda")
        rec = torch.empty((G, m, B), dtype=torch.uint8, device="cuda")
        sh.fill_synthetic(data, k, B, G, 0, 0x5E, s)
        r = {"config": tag, "k": k, "m": m, "B": B, "groups": G, "path": sh.path(k, m, B)}
        r.update(_time_ops(args, sh, torch, s, k, m, B, G, data, rec, min(k, m)))
        out.append(r)
        del data, rec
    # C3: 8192 groups (200, 32, 1400), random erasure counts 1..32 (decode only)
    k, m, B, G = 200, 32, 1400, 8192
    data = torch.empty((G, k, B), dtype=torch.uint8, device="cuda")
    rec = torch.empty((G, m, B), dtype=torch.uint8, device="cuda")
    sh.fill_synthetic(data, k, B, G, 0, 0x5E, s)
    r = {"config": "C3 random e", "k": k, "m": m, "B": B, "groups": G, "path": "fixed"}
    r.update(_time_ops(args, sh, torch, s, k, m, B, G, data, rec, 0, encode=False))
    out.append(r)
    return out


def _time_ops(args, sh, torch, s, k, m, B, G, data, rec, e_fixed, encode=True, iters=5):
    sh.encode_batch(k, m, B, G, data, rec, s)
    rows = np.zeros((G, k), np.uint8)
    es = np.zeros(G, np.int64)
    for g in range(G):
        es[g], rows[g] = sh.erasure_pattern(g, k, m, 0x5E, e_fixed)
    d_rows = torch.from_numpy(rows).cuda()
    whole = torch.cat([data, rec], dim=1)
    blocks = whole[torch.arange(G, device="cuda")[:, None], d_rows.long()]
    del whole
    emax = min(k, m)
    out = torch.empty((G, emax, B), dtype=torch.uint8, device="cuda")
    orow = torch.empty((G, emax), dtype=torch.uint8, device="cuda")
    ocnt = torch.empty(G, dtype=torch.int32, device="cuda")
    sh.batch_reserve(k, m, B, G)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    te = td = 0.0
    for it in range(iters + 1):
        if it == 1:
            sh.profile(iters)  # stage times of the timed decodes (compile-time and tile paths)
        ev[0].record()
        if encode:
            assert sh.encode_batch(k, m, B, G, data, rec, s) == 0
        ev[1].record()
        assert sh.decode_batch_out(k, m, B, G, blocks, d_rows, out, orow, ocnt, s) == 0
        ev[2].record()
        torch.cuda.synchronize()
        if it:  # first pass warms up
            te += ev[0].elapsed_time(ev[1]) / iters
            td += ev[1].elapsed_time(ev[2]) / iters
    stages = sh.profile_read()
    sh.profile(0)
    g_chk = torch.arange(G, device="cuda")[:, None]
    ok = bool(torch.equal(ocnt.cpu(), torch.from_numpy(es).int()))
    if ok and e_fixed == emax:
        ok = bool(torch.equal(out, data[g_chk, orow.long()]))
    enc_b, dec_b = G * (k + m) * B, int((k + es).sum()) * B
    r = {"decode_ms": round(td, 4), "decode_GBps": round(dec_b / td / 1e6, 1),
         "decode_frac": round(dec_b / td / 1e-3 / HBM_PEAK, 4), "mean_e": round(float(es.mean()), 2),
         "decode_ok": ok}
    if stages:
        r["decode_stages_ms"] = {"setup": round(stages[0], 4), "stageA": round(stages[1], 4), "stageB": round(stages[2], 4)}
    # work-normalized rate: the codec's work is one bitmatrix product of a B-byte block per
    # (input, output row) pair -- k*m per group for encode, k*m + e^2 for decode (stage A over all
    # m rows, stage B e x e) -- so "product_rate" = pairs x B / time in 1e15 byte-products per
    # second compares shapes with different products per byte (the headline encode: ~96)
    r["decode_product_rate"] = round((G * k * m + (es.astype(np.float64) ** 2).sum()) * B / td / 1e12, 2)
    if encode:
        r.update({"encode_ms": round(te, 4), "encode_GBps": round(enc_b / te / 1e6, 1),
                  "encode_frac": round(enc_b / te / 1e-3 / HBM_PEAK, 4),
                  "encode_product_rate": round(float(G * k * m) * B / te / 1e12, 2)})
    return r


SIMDS = 1024           # 256 CUs x 4 SIMDs
VALU_CYC = 2           # cycles per wave64 VALU instruction per SIMD at full rate (MI355X_MICROARCH.md)


def valu_leg(sq, alg_bytes, launch_ms):
    """The VALU leg of the roofline for the dominant kernel, from the SQ/GRBM pass of the
    hash-matched PMC summary (per launch): lane-ops per algorithmic byte, VALU-busy fraction
    (issue cycles per SIMD / elapsed cycles), the clock the chip held (GRBM_GUI_ACTIVE / 8 XCDs /
    this run's launch time) and the VALU-issue floor at that clock, beside the HBM floor (algorithmic
    bytes at 8 TB/s). `binding` names the larger floor."""
    if not sq or not sq.get("SQ_INSTS_VALU") or not sq.get("GRBM_GUI_ACTIVE"):
        return None
    insts, cyc = sq["SQ_INSTS_VALU"], sq["GRBM_GUI_ACTIVE"] / 8
    clock = cyc / (launch_ms * 1e-3)
    floor_ms = insts * VALU_CYC / SIMDS / clock * 1e3
    hbm_ms = alg_bytes / HBM_PEAK * 1e3
    out = {"insts_per_launch": insts, "lane_ops_per_alg_byte": round(insts * 64 / alg_bytes, 3),
           "busy_frac": round(insts * VALU_CYC / SIMDS / cyc, 4), "clock_GHz": round(clock / 1e9, 3),
           "issue_floor_ms": round(floor_ms, 4), "hbm_floor_ms": round(hbm_ms, 4),
           "binding": "valu" if floor_ms > hbm_ms else "hbm",
           "note": "counters from the profiled (rocprofv3) launches of this build; clock uses this run's "
                   "launch time, so it reads the clock under the counters' cycle count"}
    if sq.get("SQ_WAVE_CYCLES"):
        out["wait_frac"] = round(sq.get("SQ_WAIT_ANY", 0) / sq["SQ_WAVE_CYCLES"], 4)
        out["issue_stall_frac"] = round(sq.get("SQ_WAIT_INST_ANY", 0) / sq["SQ_WAVE_CYCLES"], 4)
    return out


def roofline_bound(valu, alg_bytes, launch_ms):
    """What binds the dominant kernel: "hbm" or "valu" when that floor (algorithmic bytes at 8
    TB/s; VALU issue at the held clock) is more than 0.6 of the launch, the larger one if both
    are; "latency/overlap" when neither is -- the kernel then runs well above both floors and the
    time goes to waiting and to legs that do not overlap (a label decided by a 1 %
    difference between two floors each under half the launch said nothing)."""
    hbm = alg_bytes / HBM_PEAK / (launch_ms * 1e-3)
    v = valu["issue_floor_ms"] / launch_ms if valu else 0.0
    if max(hbm, v) <= 0.6:
        return "latency/overlap"
    return "valu" if v > hbm else "hbm"


def pmc_traffic(sh, k, m, B, G, e):
    """Per-kernel HBM bytes per launch from the committed PMC summary (profiles/*/traffic*.json,
    written by tools/gpu_profile.sh: FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes,
    FETCH_SIZE doubled per the gfx950 correction). Used only when that summary was measured on
    this very library build (SHA-256; builds are deterministic, so the driver's rebuild of the
    same sources matches) and workload; else (None, None)."""
    import glob
    import hashlib
    try:
        digest = hashlib.sha256(open(sh.LIB_PATH, "rb").read()).hexdigest()
    except OSError:
        return None, None
    want = {"k": k, "m": m, "block_bytes": B, "groups": G, "erasures": e}
    here = os.path.dirname(os.path.abspath(__file__))
    for path in sorted(glob.glob(os.path.join(here, "profiles", "*", "traffic*.json")), reverse=True):
        try:
            t = json.load(open(path))
        except (OSError, ValueError):
            continue
        if t.get("lib_sha256") == digest and t.get("workload") == want:
            return t.get("kernels", {}), os.path.relpath(path, here)
    return None, None


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch(args))  # before anything touches the GPU
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        return dry_run(args, rank, world, local)
    import torch
    import torch.distributed as dist

    # rank r on GPU r; with fewer GPUs than ranks (a gloo rehearsal on one GPU) ranks share them
    dev = local % max(1, torch.cuda.device_count())
    if world > 1:
        torch.cuda.set_device(dev)
        if args.backend == "nccl":
            # a bounded collective timeout: a stuck side leg raises (and is reported) instead of
            # holding the job past the driver's limit
            import datetime
            # on a timeout the watchdog aborts the communicators but leaves the process alive
            # (torch's default kills it), so a stuck root-resident leg surfaces as an exception
            # in that leg and the main line, measured before it, still prints
            os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "2")
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev),
                                    timeout=datetime.timedelta(seconds=args.pg_timeout))
        else:
            dist.init_process_group(args.backend)
        world = dist.get_world_size()
    else:
        torch.cuda.set_device(0)
    import shorthair_amd as sh
    assert sh.lib.cauchy_256_batch_init(dev) == 0

    from shorthair_amd import dist as shd
    k, m, B, G = args.k, args.m, args.block, args.groups
    g0 = rank * G
    if args.total_groups:  # the job's groups, sharded contiguously (sizes differ by at most one)
        g0, G = shd.shard(args.total_groups, world, rank)
    emax = min(k, m)
    stream = torch.cuda.current_stream()
    s = stream.cuda_stream

    # ---- device-resident synthetic inputs (per rank: its own shard of groups) ----
    enc_in = torch.empty((G, k, B), dtype=torch.uint8, device="cuda")
    enc_out = torch.empty((G, m, B), dtype=torch.uint8, device="cuda")
    sh.fill_synthetic(enc_in, k, B, G, g0, 0xBE, s)
    sh.encode_batch(k, m, B, G, enc_in, enc_out, s)
    # decode input: each group with its erasure pattern (survivors then recovery rows)
    rows_np = np.zeros((G, k), np.uint8)
    es = np.zeros(G, np.int64)
    for g in range(G):
        es[g], rows_np[g] = sh.erasure_pattern(g0 + g, k, m, 0xBE, args.erasures)
    rows = torch.from_numpy(rows_np).cuda()
    whole = torch.cat([enc_in, enc_out], dim=1)
    dec_in = whole[torch.arange(G, device="cuda")[:, None], rows.long()].contiguous()
    del whole
    dec_out = torch.empty((G, emax, B), dtype=torch.uint8, device="cuda")
    dec_rows = torch.empty((G, emax), dtype=torch.uint8, device="cuda")
    dec_cnt = torch.empty(G, dtype=torch.int32, device="cuda")
    sh.batch_reserve(k, m, B, G)
    torch.cuda.synchronize()

    enc_bytes = G * (k + m) * B
    dec_bytes = int((k + es).sum()) * B

    def step(evs=None):
        if evs is not None:
            evs[0].record(stream)
        rc1 = sh.encode_batch(k, m, B, G, enc_in, enc_out, s)
        if evs is not None:
            evs[1].record(stream)
        rc2 = sh.decode_batch_out(k, m, B, G, dec_in, rows, dec_out, dec_rows, dec_cnt, s)
        if evs is not None:
            evs[2].record(stream)
        assert rc1 == 0 and rc2 == 0

    # correctness guard on the timed buffers (after the first settle step, and again after the
    # timed steps): the recovered blocks equal the erased originals.
    def check():
        cnt = dec_cnt.cpu().numpy()
        assert np.array_equal(cnt, es)
        g_chk = torch.arange(G, device="cuda")[:, None]
        ok = torch.equal(dec_out, enc_in[g_chk, dec_rows.long()]) if args.erasures == emax else True
        assert ok, "decode output mismatch"

    # Settle: the MI355X's power management needs ~20-30 steps (~40 ms) of sustained load after
    # any idle before the step time is steady (tools/ramp_probe.py, profiles/r06/ab_runs.txt block
    # 5: steps 0-9 from idle 1.86 ms, 10-19 1.67, 20+ 1.62-1.63). These steps are untimed like
    # the W warm-up steps that follow them, and reported in the line ("settle_steps").
    step()
    torch.cuda.synchronize()
    check()
    for _ in range(max(0, args.settle_steps - 1)):
        step()
    for i in range(args.warmup):
        step()

    # ---- timed region ----
    # Only the two HIP events around the dominant kernel (decode stage A, for the roofline) are
    # recorded in the timed steps: every event packet between the kernels costs time (measured:
    # bench.py's former three events per step plus the library's four cost 1.3 % of the step,
    # tools/step_events.py, profiles/r06/ab_runs.txt block 4). The per-op split (encode / decode,
    # setup / stage A / stage B) comes from an equal second pass recorded with every event.
    sh.profile(-args.steps)  # stage-A events of the timed decodes, no host syncs
    torch.cuda.synchronize()  # the warm-up steps (a synchronize is idle time only after them)
    if world > 1:
        dist.barrier()
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    stage_a_timed = (sh.profile_read() or (float("nan"),) * 3)[1]
    # ---- breakdown pass (not timed for the headline) ----
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    sh.profile(args.steps)
    torch.cuda.synchronize()
    for i in range(args.steps):
        step(evs[i])
    torch.cuda.synchronize()
    enc_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
    dec_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in evs]))
    stages = list(sh.profile_read() or (float("nan"),) * 3)
    stages_breakdown_a = stages[1]
    stages[1] = stage_a_timed  # the roofline's launch time: measured live in the timed steps
    sh.profile(0)
    check()
    elapsed = shd.max_over_ranks(elapsed, device="cuda")
    dec_bytes_all = shd.sum_over_ranks(dec_bytes, device="cuda")

    # ---- root-resident variant (N > 1): groups start and end on rank 0's GPU; one RCCL scatter of
    # the data shards over xGMI, encode on every GPU, one RCCL gather of the recovery shards.
    # Reported beside the main line, never as `value`.
    # (the main line's last collective runs before the side leg: a failed leg leaves the process
    # group unusable, and the line must still print)
    enc_bytes_all = shd.sum_over_ranks(enc_bytes, device="cuda")
    root_res = None
    pg_ok = True
    if world > 1 and args.root_steps > 0:
        try:
            root_res = root_resident(args, sh, shd, dist, torch, rank, world, G, k, m, B, s, enc_in, enc_out,
                                     dec_in, rows, dec_out, dec_rows, dec_cnt, es)
        except Exception as exc:  # never lose the main line over the side measurement
            root_res = {"error": f"{type(exc).__name__}: {exc}"}
            pg_ok = False
    total = (enc_bytes_all + dec_bytes_all) * args.steps
    value = total / elapsed / 2**30
    ms_per_step = elapsed / args.steps * 1e3

    if rank == 0:
        enc_bw = enc_bytes / (enc_ms * 1e-3)
        dec_bw = dec_bytes / (dec_ms * 1e-3)
        kb = G * (k + m) * B  # algorithmic bytes per launch of either compile-time kernel
        a_ms = stages[1]
        dom = (("encode kernel", enc_ms) if not (a_ms > enc_ms) else ("decode stage-A kernel", a_ms))
        pmc, traffic_src = pmc_traffic(sh, k, m, B, G, args.erasures)
        names = {"encode": f"sh::fixed::kern_k{k}_m{m}_enc", "decode_stageA": f"sh::fixed::kern_k{k}_m{m}_dec",
                 "decode_stageB": "sh::stageb_v2"}
        e_all = int(es.sum())
        # stage A reads the k received blocks (survivors + recovery rows) and writes m residual
        # rows, like encode; stage B reads e residual rows and writes e recovered blocks
        alg = {"encode": kb, "decode_stageA": kb, "decode_stageB": 2 * e_all * B}
        traffic = None
        valu = None
        pmc_line = None
        if pmc:
            pmc_line = {}
            def find(nm):  # rocprofv3 names templates as "void sh::stageb_v2<4>(sh::StageBV2Args)"
                return next((v for key, v in pmc.items() if key == nm or key.split("(")[0].split(" ")[-1].split("<")[0] == nm), None)
            for op, nm in names.items():
                t = find(nm)
                if t is not None:
                    pmc_line[op] = {"read_bytes": t["read_bytes"], "write_bytes": t["write_bytes"],
                                    "alg_bytes": alg[op], "traffic_over_alg": round(t["hbm_bytes"] / alg[op], 3)}
            dom_op = "encode" if dom[0].startswith("encode") else "decode_stageA"
            traffic = (find(names[dom_op]) or {}).get("hbm_bytes")
            valu = valu_leg((find(names[dom_op]) or {}).get("sq"), kb, dom[1])
        threads = args.cpu_threads or host_cores()
        cpu = None if args.no_cpu else cpu_baseline(k, m, B, args.erasures, args.cpu_seconds, threads)
        line = {
            "metric": "cauchy_256 encode+decode GiB/s (device-resident), k=200 m=32 ×1400B; %HBM peak",
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle_steps": args.settle_steps,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.total_groups else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (PCG32 per block, device-generated; erasure patterns PCG32)",
            "config": {"workload": (f"{args.total_groups} groups over {world} GPUs" if args.total_groups else
                                    f"{G} groups/GPU") + f" encode + decode, k={k} m={m} "
                                   f"B={B} e={args.erasures or 'rand'}",
                       "k": k, "m": m, "block_bytes": B, "groups_per_gpu": G,
                       "total_groups": args.total_groups or G * world,
                       "erasures": args.erasures, "parallelism": f"groups sharded x{world}"},
            "hbm_frac": round(value * 2**30 / world / HBM_PEAK, 4),
            "payload_GiBps": round(enc_bytes_all / (k + m) * k * 2 * args.steps / elapsed / 2**30, 3),
            "ops": {"encode_ms": round(enc_ms, 4), "encode_GBps": round(enc_bw / 1e9, 1),
                    "decode_ms": round(dec_ms, 4), "decode_GBps": round(dec_bw / 1e9, 1),
                    "decode_setup_ms": round(stages[0], 4), "decode_stageA_ms": round(stages[1], 4),
                    "decode_stageB_ms": round(stages[2], 4),
                    # encode / decode / setup / stage B: the breakdown pass (every event recorded);
                    # stage A: the timed steps' own events (its breakdown-pass time beside it)
                    "decode_stageA_breakdown_ms": round(stages_breakdown_a, 4),
                    "timing": "headline steps carry only the stage-A event pair; per-op times from an equal breakdown pass"},
            "roofline": {"bound": roofline_bound(valu, kb, dom[1]), "kernel": dom[0],
                         "achieved": round(kb / (dom[1] * 1e-3) / 1e9, 1),
                         "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                         "frac": round(kb / (dom[1] * 1e-3) / HBM_PEAK, 4), "traffic": traffic,
                         "traffic_source": traffic_src,
                         "traffic_over_alg": round(traffic / kb, 3) if traffic else None,
                         "alg_bytes_per_launch": kb, "launch_ms": round(dom[1], 4),
                         # the two floors as fractions of this launch, top-level scalars (VERDICT r4
                         # #4: the nested `valu` dict did not survive into the driver's record)
                         "hbm_floor_frac": round(kb / HBM_PEAK / (dom[1] * 1e-3), 4),
                         "valu_floor_frac": round(valu["issue_floor_ms"] / dom[1], 4) if valu else None,
                         "valu_busy": valu["busy_frac"] if valu else None,
                         "wait_frac": valu.get("wait_frac") if valu else None,
                         "valu": valu},
            "op_roofline": {  # algorithmic bytes / measured time, as a fraction of 8 TB/s
                "encode": round(enc_bytes / (enc_ms * 1e-3) / HBM_PEAK, 4),
                "decode": round(dec_bytes / (dec_ms * 1e-3) / HBM_PEAK, 4),
                "decode_stageA": round(alg["decode_stageA"] / (stages[1] * 1e-3) / HBM_PEAK, 4),
                "decode_stageB": round(alg["decode_stageB"] / (stages[2] * 1e-3) / HBM_PEAK, 4)},
            "pmc_traffic": pmc_line,
            "cpu_baseline": cpu,
        }
        if root_res is not None:
            line["root_resident"] = root_res
        if not args.no_sweep and world == 1:
            try:
                line["sweep"] = sweep(args, sh, torch, s)
            except Exception as exc:  # a side measurement never loses the main line
                line["sweep"] = {"error": f"{type(exc).__name__}: {exc}"}
        if args.host_calls > 0 and world == 1:
            try:
                line["host_path"] = host_path(args, sh, torch, k, m, B, s)
            except Exception as exc:  # a side measurement never loses the main line
                line["host_path"] = {"error": f"{type(exc).__name__}: {exc}"}
        print(json.dumps(line), flush=True)
    if world > 1:
        try:
            if pg_ok:
                dist.destroy_process_group()
        except Exception:  # teardown after a failed side leg: the line is already out
            pass


if __name__ == "__main__":
    main()
