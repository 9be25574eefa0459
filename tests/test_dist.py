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
