"""Multi-process (world size 2, gloo, CPU) tests of the N>1 plumbing: group sharding, the
max-over-ranks / sum-over-ranks timing reductions bench.py uses, and the root-resident
scatter / gather of group shards (shorthair_amd/dist.py). The GPU box runs the same code on
RCCL; the codec calls themselves need a GPU and are covered by test_gpu_parity.py."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp



def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from shorthair_amd import dist as d
        out = {}
        # sharding covers [0, total) exactly, contiguous, sizes within one
        total = 8193
        g0, n = d.shard(total, world, rank)
        out["shard"] = (g0, n)
        # reductions
        out["max"] = d.max_over_ranks(1.5 + rank)
        out["sum"] = d.sum_over_ranks(10 * (rank + 1))
        # root-resident scatter / gather of [world*G][k][B] uint8 groups
        G, k, B = 3, 4, 24
        root = None
        if rank == 0:
            root = torch.from_numpy(np.arange(world * G * k * B, dtype=np.int64).astype(np.uint8)
                                    .reshape(world * G, k, B))
        mine = torch.empty((G, k, B), dtype=torch.uint8)
        d.scatter_groups(mine, root, root=0)
        out["scattered_ok"] = bool(
            np.array_equal(mine.numpy(), (np.arange(world * G * k * B, dtype=np.int64).astype(np.uint8)
                                          .reshape(world * G, k, B))[rank * G:(rank + 1) * G]))
        # "recovery" = shard ^ 0x5A, gathered back on the root
        rec = mine ^ 0x5A
        back = torch.empty((world * G, k, B), dtype=torch.uint8) if rank == 0 else None
        d.gather_groups(rec, back, root=0)
        if rank == 0:
            out["gathered_ok"] = bool(np.array_equal(back.numpy(), root.numpy() ^ 0x5A))
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_world2_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    shards = sorted(res[r]["shard"] for r in range(world))
    assert shards[0][0] == 0 and shards[-1][0] + shards[-1][1] == 8193
    assert shards[0][0] + shards[0][1] == shards[1][0]
    assert abs(shards[0][1] - shards[1][1]) <= 1
    for r in range(world):
        assert res[r]["max"] == 2.5
        assert res[r]["sum"] == 30.0
        assert res[r]["scattered_ok"]
    assert res[0]["gathered_ok"]


@pytest.mark.parametrize("total,world", [(8192, 8), (7, 3), (1, 4), (0, 2)])
def test_shard_partition(total, world):
    from shorthair_amd import dist as d
    got = [d.shard(total, world, r) for r in range(world)]
    pos = 0
    for g0, n in got:
        assert g0 == pos and n >= 0
        pos += n
    assert pos == total
    assert max(n for _, n in got) - min(n for _, n in got) <= 1


def _stream_worker(rank, world, port, q, total, chunk, overlap):
    """shd.RootStream at C5's shape, scaled down: the root holds one [world * chunk] window per
    tensor; every rank's shard (uneven when total % world != 0) arrives in chunks -- two input
    tensors, like decode's received blocks + row arrays -- and its outputs (three tensors, like
    decode's recovered blocks + rows + counts) go back through the root's output windows. With
    overlap, chunk j+1's scatter is in flight while chunk j computes."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from shorthair_amd import dist as d
        k, B = 3, 16
        sizes = [d.shard(total, world, r)[1] for r in range(world)]
        if chunk is None:  # the default: every rank derives the same chunk from max(sizes)
            chunk = d.root_chunk_size(sizes, k * B, window_bytes=world * 4 * k * B)
        g0, G = d.shard(total, world, rank)

        def group_bytes(g):  # the root's content for global group g
            return (np.arange(k * B, dtype=np.int64) * 7 + g * 131).astype(np.uint8).reshape(k, B)

        blocks = torch.zeros((G, k, B), dtype=torch.uint8)
        rows = torch.zeros((G, k), dtype=torch.uint8)
        out = torch.zeros((G, 2, B), dtype=torch.uint8)
        orow = torch.zeros((G, 2), dtype=torch.uint8)
        cnt = torch.zeros(G, dtype=torch.int32)
        rs = d.RootStream(sizes, chunk, [blocks, rows], [out, orow, cnt])
        seen = []

        def compute(lo, n):
            seen.append((lo, n))
            out[lo:lo + n] = blocks[lo:lo + n, :2] ^ 0x5A
            orow[lo:lo + n] = rows[lo:lo + n, :2] + 1
            cnt[lo:lo + n] = rows[lo:lo + n, 0].int() * 3

        # the root's per-chunk windows (a real feeder refills double-buffered windows per chunk)
        win_in = win_out = None
        if rank == 0:
            win_in, win_out = {}, {}
            for j in range(rs.nchunks):
                win_in[j] = [torch.zeros((world * chunk, k, B), dtype=torch.uint8),
                             torch.zeros((world * chunk, k), dtype=torch.uint8)]
                win_out[j] = [torch.zeros((world * chunk, 2, B), dtype=torch.uint8),
                              torch.zeros((world * chunk, 2), dtype=torch.uint8),
                              torch.zeros(world * chunk, dtype=torch.int32)]
                for r in range(world):
                    rg0, rn = d.shard(total, world, r)
                    for i in range(max(0, min(chunk, rn - j * chunk))):
                        g = rg0 + j * chunk + i
                        win_in[j][0][r * chunk + i] = torch.from_numpy(group_bytes(g))
                        win_in[j][1][r * chunk + i] = torch.tensor([g % 256, 1, 2], dtype=torch.uint8)
        rs.run(compute, win_in and win_in.__getitem__, win_out and win_out.__getitem__, overlap=overlap)
        back_ok = True
        if rank == 0:
            for j in range(rs.nchunks):
                for r, a, n in rs.slots(j):
                    rg0 = d.shard(total, world, r)[0]
                    for i in range(n):
                        g = rg0 + j * chunk + i
                        back_ok &= bool(np.array_equal(win_out[j][0][a + i].numpy(), group_bytes(g)[:2] ^ 0x5A))
                        back_ok &= win_out[j][1][a + i].tolist() == [(g % 256) + 1, 2]
                        back_ok &= int(win_out[j][2][a + i]) == (g % 256) * 3
        ok = all(np.array_equal(blocks[i].numpy(), group_bytes(g0 + i)) for i in range(G))
        ok &= sorted(seen) == [(lo, min(chunk, G - lo)) for lo in range(0, G, chunk)]
        q.put((rank, {"ok": ok, "back_ok": back_ok, "chunks": rs.nchunks, "G": G, "chunk": chunk}))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,total,chunk,overlap", [(2, 11, 4, True), (3, 10, 3, True), (3, 9, 5, True),
                                                       (2, 11, 4, False), (3, 13, None, True),
                                                       (2, 3, 1, True)])
def test_root_stream(world, total, chunk, overlap):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stream_worker, args=(r, world, port, q, total, chunk, overlap))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sum(res[r]["G"] for r in range(world)) == total
    assert len({res[r]["chunk"] for r in range(world)}) == 1  # every rank agrees on the chunk
    for r in range(world):
        assert res[r]["ok"], r
        assert res[r]["chunks"] == -(-max(res[x]["G"] for x in range(world)) // res[r]["chunk"])
    assert res[0]["back_ok"]


def test_c5_total_groups_and_root_window():
    """bench.py --gpus 8 --total-groups 1048576: 131,072 groups per rank; the root-resident leg's
    window at (200, 32, 1400) stays within ~16 GB of the root's HBM (the whole batch is 325 GB)."""
    from shorthair_amd import dist as d
    sizes = [d.shard(1 << 20, 8, r)[1] for r in range(8)]
    assert sizes == [131072] * 8
    chunk = d.root_chunk_size(sizes, (200 + 32) * 1400)
    assert 8 * chunk * (200 + 32) * 1400 <= 16e9 and chunk >= 4096
    assert d.chunk_count(sizes, chunk) * chunk >= 131072
    assert d.root_chunk_size([100, 100], (200 + 32) * 1400) == 100  # small batches: one chunk
    # uneven shards: the chunk follows the largest shard on every rank
    assert d.root_chunk_size([51, 50], 10, window_bytes=1e9) == 51
