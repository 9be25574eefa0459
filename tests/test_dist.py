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


def _chunk_worker(rank, world, port, q, total, chunk):
    """Streamed root-resident pass (bench.py root_resident at C5 scale, scaled down): the root
    holds one [world * chunk] window; every rank's shard (uneven: total % world != 0) arrives in
    chunks and its "recovery" (shard ^ 0x5A, one row per group) goes back through the window."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from shorthair_amd import dist as d
        k, B = 3, 16
        sizes = [d.shard(total, world, r)[1] for r in range(world)]
        g0, G = d.shard(total, world, rank)
        n_chunks = d.chunk_count(sizes, chunk)

        def group_bytes(g):  # the root's content for global group g
            return (np.arange(k * B, dtype=np.int64) * 7 + g * 131).astype(np.uint8).reshape(k, B)

        mine = torch.zeros((G, k, B), dtype=torch.uint8)
        rec = torch.zeros((G, 1, B), dtype=torch.uint8)
        st_in = torch.empty((chunk, k, B), dtype=torch.uint8)
        st_out = torch.empty((chunk, 1, B), dtype=torch.uint8)
        win_in = torch.empty((world * chunk, k, B), dtype=torch.uint8) if rank == 0 else None
        win_out = torch.empty((world * chunk, 1, B), dtype=torch.uint8) if rank == 0 else None
        back_ok = True
        for j in range(n_chunks):
            if rank == 0:  # the root refills its window with chunk j of every rank's shard
                win_in.zero_()
                for r in range(world):
                    rg0, rn = d.shard(total, world, r)
                    for i in range(max(0, min(chunk, rn - j * chunk))):
                        win_in[r * chunk + i] = torch.from_numpy(group_bytes(rg0 + j * chunk + i))
            n = d.scatter_chunk(mine, j, chunk, win_in, st_in)
            lo = j * chunk
            rec[lo:lo + n] = mine[lo:lo + n, :1] ^ 0x5A
            d.gather_chunk(rec, j, chunk, win_out, st_out)
            if rank == 0:
                for r in range(world):
                    rg0, rn = d.shard(total, world, r)
                    for i in range(max(0, min(chunk, rn - j * chunk))):
                        want = group_bytes(rg0 + j * chunk + i)[:1] ^ 0x5A
                        back_ok &= bool(np.array_equal(win_out[r * chunk + i].numpy(), want))
        ok = all(np.array_equal(mine[i].numpy(), group_bytes(g0 + i)) for i in range(G))
        q.put((rank, {"ok": ok, "back_ok": back_ok, "chunks": n_chunks, "G": G}))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,total,chunk", [(2, 11, 4), (3, 10, 3), (3, 9, 5)])
def test_chunked_root_scatter_gather(world, total, chunk):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_chunk_worker, args=(r, world, port, q, total, chunk)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sum(res[r]["G"] for r in range(world)) == total
    for r in range(world):
        assert res[r]["ok"], r
        assert res[r]["chunks"] == -(-max(res[x]["G"] for x in range(world)) // chunk)
    assert res[0]["back_ok"]


def test_c5_total_groups_and_root_window():
    """bench.py --gpus 8 --total-groups 1048576: 131,072 groups per rank; the root-resident leg's
    window at (200, 32, 1400) stays within ~16 GB of the root's HBM (the whole batch is 325 GB)."""
    import importlib.util
    from shorthair_amd import dist as d
    spec = importlib.util.spec_from_file_location("bench", os.path.join(os.path.dirname(__file__), "..", "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    sizes = [d.shard(1 << 20, 8, r)[1] for r in range(8)]
    assert sizes == [131072] * 8
    chunk = bench.root_window_chunk(8, 131072, 200, 32, 1400)
    assert 8 * chunk * (200 + 32) * 1400 <= 16e9 and chunk >= 4096
    assert d.chunk_count(sizes, chunk) * chunk >= 131072
    assert bench.root_window_chunk(2, 100, 200, 32, 1400) == 100  # small batches: one chunk
