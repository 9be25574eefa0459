"""Multi-GPU plumbing for batches of code groups.

Code groups are independent (no state crosses groups, reference cauchy_256.cpp keeps none
between calls), so N GPUs each code a contiguous shard of groups with no collective on the data
path ("weak scaling", bench.py's default). When the groups start and end on one root GPU
(north_star: "RCCL over xGMI only to scatter input shards and gather recovery shards"),
`scatter_groups` / `gather_groups` move the shards with one RCCL scatter / gather each -- a
single large collective per batch, the xGMI-friendly shape (7 point-to-point links from the
root; no ring reduction involved).

Everything here is torch.distributed on whatever backend the process group uses: "nccl" (RCCL)
on the GPU box, "gloo" for the CPU tests (tests/test_dist.py, world size 2).
"""
import torch
import torch.distributed as dist


def shard(total_groups, world, rank):
    """Contiguous shard (first group, group count) of rank: sizes differ by at most one."""
    base, extra = divmod(total_groups, world)
    g0 = rank * base + min(rank, extra)
    return g0, base + (1 if rank < extra else 0)


def max_over_ranks(x, device=None):
    """Max of a float over all ranks (the slowest rank sets a step's time)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x, device=None):
    """Sum of a float over all ranks (aggregate bytes moved by the job)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def scatter_groups(shard_out, root_batch=None, root=0):
    """Root's [world * G][...] batch -> every rank's [G][...] shard (equal shards).

    One collective: dist.scatter of the root's contiguous per-rank slices."""
    world = dist.get_world_size()
    if dist.get_rank() == root:
        assert root_batch is not None and root_batch.shape[0] == world * shard_out.shape[0]
        chunks = list(root_batch.chunk(world, dim=0))
        dist.scatter(shard_out, chunks, src=root)
    else:
        dist.scatter(shard_out, None, src=root)
    return shard_out


def gather_groups(shard_in, root_batch=None, root=0):
    """Every rank's [G][...] shard -> root's [world * G][...] batch (equal shards)."""
    world = dist.get_world_size()
    if dist.get_rank() == root:
        assert root_batch is not None and root_batch.shape[0] == world * shard_in.shape[0]
        chunks = list(root_batch.chunk(world, dim=0))
        dist.gather(shard_in, chunks, dst=root)
    else:
        dist.gather(shard_in, None, dst=root)
    return root_batch
