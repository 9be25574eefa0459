"""Multi-GPU plumbing for batches of code groups.

Code groups are independent (no state crosses groups, reference cauchy_256.cpp keeps none
between calls), so N GPUs each code a contiguous shard of groups with no collective on the data
path ("weak scaling", bench.py's default). When the groups start and end on one root GPU
(north_star: "RCCL over xGMI only to scatter input shards and gather recovery shards"),
`scatter_groups` / `gather_groups` move the shards with one RCCL scatter / gather each -- a
single large collective per batch, the xGMI-friendly shape (7 point-to-point links from the
root; no ring reduction involved). `RootStream` streams a batch larger than one GPU through a
window on the root, chunk by chunk, with the scatter of the next chunk and the gather of the
previous one overlapping each chunk's kernels (bench.py's root-resident leg, encode and decode).

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


def root_chunk_size(sizes, per_group_bytes, window_bytes=16e9):
    """Groups per rank per chunk of a root-resident pass. Computed from max(sizes), which every
    rank knows, so all ranks agree on it even when the shards differ in size (a chunk sized from
    each rank's own shard would make the root scatter world * chunk0 slices while another rank
    posts chunk1-sized buffers: gloo raises, RCCL hangs). The root's window of world * chunk
    groups stays within `window_bytes`."""
    world = len(sizes)
    biggest = max(sizes) if sizes else 0
    return int(max(1, min(biggest, window_bytes // (world * per_group_bytes))))


def _coll_scatter(dst, win, root, async_op):
    if dist.get_rank() == root:
        return dist.scatter(dst, list(win.chunk(dist.get_world_size(), dim=0)), src=root, async_op=async_op)
    return dist.scatter(dst, None, src=root, async_op=async_op)


def _coll_gather(src, win, root, async_op):
    if dist.get_rank() == root:
        return dist.gather(src, list(win.chunk(dist.get_world_size(), dim=0)), dst=root, async_op=async_op)
    return dist.gather(src, None, dst=root, async_op=async_op)


class RootStream:
    """Streamed root-resident pass with the collectives overlapped.

    The root holds one window of world x chunk groups per tensor; every rank's shard passes
    through it chunk by chunk: one scatter per input tensor (e.g. decode: received blocks + row
    arrays), `compute(lo, n)` on the rank's groups [lo, lo + n), one gather per output tensor
    (decode: recovered blocks + their rows + counts) back into the root's window. Chunk j+1's
    scatter is posted before chunk j computes and chunk j's gather is posted right after it
    (async_op), so on RCCL both run on the communicator's stream under the codec kernels: the
    communicator stream waits for the compute stream only at each collective's issue point, and
    the compute stream waits (Work.wait) only for the chunk it is about to code.

    A rank whose shard ends inside a chunk (or before it) receives into / sends from one of two
    stage buffers (alternating, so a posted scatter never writes the stage the previous chunk is
    still copying out of); a gather's stage is reused only after that gather completed."""

    def __init__(self, sizes, chunk, ins, outs, root=0):
        self.world, self.rank, self.root = dist.get_world_size(), dist.get_rank(), root
        assert len(sizes) == self.world and chunk > 0
        self.sizes, self.chunk = list(sizes), chunk
        self.G = self.sizes[self.rank]
        self.nchunks = chunk_count(self.sizes, chunk)
        self.ins, self.outs = ins, outs
        for t in list(ins) + list(outs):
            assert t.shape[0] == self.G and t.is_contiguous()
        short = self.G < self.nchunks * chunk
        self.st_in = [[t.new_empty((chunk,) + tuple(t.shape[1:])) for t in ins] for _ in range(2)] if short else None
        self.st_out = [[t.new_zeros((chunk,) + tuple(t.shape[1:])) for t in outs] for _ in range(2)] if short else None

    def _n(self, j):
        return max(0, min(self.chunk, self.G - j * self.chunk))

    def run(self, compute, win_in=None, win_out=None, overlap=True):
        """One pass over every chunk. win_in / win_out (the root only; None elsewhere): its
        [world * chunk][...] windows, one per input / output tensor -- a list (the same window
        for every chunk) or a callable j -> list (a real feeder refilling double-buffered windows
        per chunk; a window must stay untouched until its collective completed)."""
        C, root = self.chunk, self.root
        nin, nout = len(self.ins), len(self.outs)
        if self.rank == root:
            def windows(w, ts):
                def get(j):
                    ws = w(j) if callable(w) else w
                    assert len(ws) == len(ts)
                    for x, t in zip(ws, ts):
                        assert x.shape[0] == self.world * C and x.shape[1:] == t.shape[1:] and x.dtype == t.dtype
                    return ws
                return get
            get_in, get_out = windows(win_in, self.ins), windows(win_out, self.outs)
        else:
            get_in, get_out = (lambda j: [None] * nin), (lambda j: [None] * nout)
        posted, gathers = {}, {}

        def post_scatter(j):
            n, lo = self._n(j), j * C
            dsts = [t[lo:lo + C] for t in self.ins] if n == C else self.st_in[j % 2]
            works = [_coll_scatter(d, w, root, overlap) for d, w in zip(dsts, get_in(j))]
            posted[j] = (works, dsts, n, lo)

        def finish_scatter(j):
            works, dsts, n, lo = posted.pop(j)
            for w in works:
                if w is not None:
                    w.wait()
            if n and n < C:
                for t, d in zip(self.ins, dsts):
                    t[lo:lo + n].copy_(d[:n])
            return n, lo

        def post_gather(j, n, lo):
            if n == C:
                srcs = [t[lo:lo + C] for t in self.outs]
            else:
                prev = gathers.pop(j - 2, None)  # the last gather that read this stage
                for w in prev or ():
                    if w is not None:
                        w.wait()
                srcs = self.st_out[j % 2]
                for t, s in zip(self.outs, srcs):
                    s.zero_()
                    if n:
                        s[:n].copy_(t[lo:lo + n])
            gathers[j] = [_coll_gather(s, w, root, overlap) for s, w in zip(srcs, get_out(j))]

        if self.nchunks:
            post_scatter(0)
        for j in range(self.nchunks):
            if overlap and j + 1 < self.nchunks:
                post_scatter(j + 1)
            n, lo = finish_scatter(j)
            if n:
                compute(lo, n)
            post_gather(j, n, lo)
            if not overlap and j + 1 < self.nchunks:
                post_scatter(j + 1)
        for works in gathers.values():
            for w in works:
                if w is not None:
                    w.wait()

    def slots(self, j=None):
        """(rank, first window row, groups) of every rank's data in the window after chunk j
        (default: the last chunk)."""
        j = self.nchunks - 1 if j is None else j
        return [(r, r * self.chunk, max(0, min(self.chunk, n - j * self.chunk))) for r, n in enumerate(self.sizes)]
