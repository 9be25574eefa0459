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


def chunk_count(shard_sizes, chunk):
    """Chunks a chunked root-resident pass needs: every rank's shard in pieces of `chunk` groups."""
    return max(0, -(-max(shard_sizes) // chunk)) if shard_sizes and chunk > 0 else 0


def scatter_chunk(shard_out, j, chunk, root_chunk=None, stage=None, root=0):
    """Chunk j of a streamed scatter: the root's [world * chunk][...] window -> groups
    [j*chunk, j*chunk + chunk) of every rank's shard (fewer for a rank whose shard ends inside the
    chunk: it receives into `stage`, a [chunk][...] buffer, and keeps what its shard holds).

    For batches larger than the root GPU (C5: 1M groups of (200, 32, 1400) = 280 GB of input),
    the root only ever holds one window; each chunk is one RCCL scatter over xGMI.
    Returns the number of groups this rank received into its shard."""
    world = dist.get_world_size()
    lo = j * chunk
    n = max(0, min(chunk, shard_out.shape[0] - lo))
    full = n == chunk
    dst = shard_out[lo:lo + chunk] if full else stage
    assert dst is not None and dst.shape[0] == chunk, "a partial chunk needs a [chunk] stage buffer"
    if dist.get_rank() == root:
        assert root_chunk is not None and root_chunk.shape[0] == world * chunk
        dist.scatter(dst, list(root_chunk.chunk(world, dim=0)), src=root)
    else:
        dist.scatter(dst, None, src=root)
    if not full and n > 0:
        shard_out[lo:lo + n].copy_(stage[:n])
    return n


def gather_chunk(shard_in, j, chunk, root_chunk=None, stage=None, root=0):
    """Chunk j of a streamed gather: groups [j*chunk, j*chunk + chunk) of every rank's shard ->
    the root's [world * chunk][...] window (rank r's groups at [r*chunk, r*chunk + n_r); a
    partial chunk is sent from `stage`, zero-padded). Returns this rank's group count."""
    world = dist.get_world_size()
    lo = j * chunk
    n = max(0, min(chunk, shard_in.shape[0] - lo))
    if n == chunk:
        src = shard_in[lo:lo + chunk]
    else:
        assert stage is not None and stage.shape[0] == chunk
        src = stage
        src.zero_()
        if n > 0:
            src[:n].copy_(shard_in[lo:lo + n])
    if dist.get_rank() == root:
        assert root_chunk is not None and root_chunk.shape[0] == world * chunk
        dist.gather(src, list(root_chunk.chunk(world, dim=0)), dst=root)
    else:
        dist.gather(src, None, dst=root)
    return n
