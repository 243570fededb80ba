"""Multi-GPU all-pairs histogram: one process per GPU, RCCL all-reduce of the counts.

The unordered pairs of a code set are cut into ``items`` equal work items (row block
x column chunk, see sctools_amd/csrc/allpairs.hip).  Rank r of W counts the
contiguous item range ``item_range(items, r, W)`` on its own GPU against its own
replica of the codes (a few MB, so every rank holds them all) and, in the MOMENTS
scheme, moment share r of W, producing ``ncounts`` uint64 counts.  The counts are
linear in the pairs, so ONE all-reduce(sum) of ``ncounts`` int64 over RCCL
(torch.distributed backend "nccl" on ROCm) combines the ranks; every rank then
inverts the summed counts to the exact histogram.  Integer sums are order
independent, so the result is bit-identical for any W.

Nearest-whitelist correction (config 4) and the batch encoder split their records into
contiguous ranges per rank with the whitelist replicated; ``gather_ranges`` all-gathers
the per-rank results (no reduction).

The reference (barcode.py:39-46) has no parallelism at all; this is new.
"""

import numpy as np

from . import _lib

__all__ = ["item_range", "combine_counts", "allpairs_histogram_sharded", "gather_ranges", "nearest_sharded",
           "encode_sharded"]


def item_range(items, rank, world):
    """Contiguous, balanced shard [begin, end) of [0, items) for `rank` of `world`."""
    if not 0 <= rank < world:
        raise ValueError("rank %d outside world of %d" % (rank, world))
    return items * rank // world, items * (rank + 1) // world


def combine_counts(counts, group=None, scheme=_lib.SCHEME_SUBSETS, nbins=None):
    """Sum per-rank counts (a torch int64 tensor, in place) over the process group and
    return the exact histogram as np.uint64 on every rank."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(counts, op=dist.ReduceOp.SUM, group=group)
    host = counts.detach().cpu().numpy().astype(np.int64).view(np.uint64)
    return _lib.counts_to_hist(host, scheme, nbins)


def allpairs_histogram_sharded(codes, code_bits=None, group=None, device=None, stream=None):
    """Histogram of TwoBit distances over all unordered pairs of `codes` (np.uint64 or a
    torch tensor), sharded over the ranks of `group` (one GPU each).  Call on every rank
    with the same codes."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    device = device or torch.device("cuda", torch.cuda.current_device())
    if isinstance(codes, np.ndarray):
        d_codes = torch.from_numpy(np.ascontiguousarray(codes, dtype=np.uint64).view(np.int64)).to(device)
    else:
        d_codes = codes.to(device=device, dtype=torch.int64).contiguous()
    n = int(d_codes.numel())
    if code_bits is None:
        orv = int(np.bitwise_or.reduce(d_codes.cpu().numpy().view(np.uint64))) if n else 0
        code_bits = max(1, orv.bit_length())
    plan = _lib.AllPairsPlan(d_codes.data_ptr(), n, code_bits)
    try:
        s = (stream or torch.cuda.current_stream(device)).cuda_stream
        b, e = item_range(plan.items, rank, world)
        counts = torch.zeros(plan.ncounts, dtype=torch.int64, device=device)
        plan.build(s, b, e)  # only the column chunks of this rank's items
        plan.moments(counts.data_ptr(), rank, world, s)
        plan.count(counts.data_ptr(), b, e, 0, s)
        return combine_counts(counts, group, plan.scheme, plan.nbins)
    finally:
        plan.close()


def _group_info(group):
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


def gather_ranges(local, n, group=None):
    """All-gather the per-rank contiguous slices ``[item_range(n, r, W)]`` (along the first
    axis) of a numpy array into the whole array, on every rank (config 4 and
    the encoder split their records into contiguous ranges with no reduction; this is the
    only exchange).  ``None`` passes through."""
    import torch
    import torch.distributed as dist
    if local is None:
        return None
    world, rank = _group_info(group)
    local = np.ascontiguousarray(local)
    if world == 1:
        return local
    sizes = [item_range(n, r, world)[1] - item_range(n, r, world)[0] for r in range(world)]
    assert local.shape[0] == sizes[rank], (local.shape, sizes[rank])
    row = local.dtype.itemsize * int(np.prod(local.shape[1:], dtype=np.int64))
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
    # bytes on the wire: any dtype and row shape, padded to the largest slice
    raw = np.zeros(max(sizes) * row, dtype=np.uint8)
    raw[: local.nbytes] = local.reshape(-1).view(np.uint8)
    mine = torch.from_numpy(raw).to(dev)
    parts = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine, group=group)
    return np.concatenate([p.cpu().numpy()[: s * row].view(local.dtype).reshape((s,) + local.shape[1:])
                           for p, s in zip(parts, sizes)])


def nearest_sharded(kind, whitelist, queries, max_d=1, code_bits=None, group=None, fn=None):
    """Nearest-whitelist correction with the queries split into contiguous ranges, one per
    rank (the whitelist replicated); returns the whole (index, dist) on every rank.  ``fn``
    is the per-rank computation (default: the GPU path, ``_lib.nearest``)."""
    world, rank = _group_info(group)
    q = np.ascontiguousarray(queries, dtype=np.uint64).reshape(-1)
    b, e = item_range(q.size, rank, world)
    idx, dist_ = (fn or _lib.nearest)(kind, whitelist, q[b:e], max_d, code_bits)
    return gather_ranges(np.asarray(idx, dtype=np.int32), q.size, group), \
        gather_ranges(np.asarray(dist_, dtype=np.uint8), q.size, group)


def encode_sharded(kind, seqs, L, group=None, fn=None):
    """TwoBit / ThreeBit batch encode with the records split into contiguous ranges, one per
    rank; returns what ``fn`` (default ``_lib.encode``: codes, gc, flags) returns, gathered
    over the ranks."""
    world, rank = _group_info(group)
    seqs = np.asarray(seqs)
    b, e = item_range(len(seqs), rank, world)
    outs = (fn or _lib.encode)(kind, seqs[b:e], L)
    return tuple(gather_ranges(None if o is None else np.asarray(o), len(seqs), group) for o in outs)
