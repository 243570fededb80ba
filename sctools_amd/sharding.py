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
contiguous ranges per rank with the whitelist replicated and no collective:
each rank reads only its own range of the input and keeps its own slice of the results.
``gather_ranges`` (opt-in) all-gathers the slices when a caller wants the whole result
on every rank.

The reference (barcode.py:39-46) has no parallelism at all; this is new.
"""

import numpy as np

from . import _lib

__all__ = ["item_range", "combine_counts", "ShardedAllPairs", "allpairs_histogram_sharded", "gather_ranges", "nearest_sharded",
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


class ShardedAllPairs:
    """One rank's share of ``Barcodes.summarize_hamming_distances`` (barcode.py:39-46) on
    its own GPU: a plan over this rank's replica of the codes, the rank's item range
    ``item_range(items, rank, W)`` (SPECTRAL: transform slices; pair schemes: row block x
    column chunk items plus moment share r of W), and the one all-reduce of the counts.

    ``step()`` is the whole per-rank hot path -- build, count, all-reduce (W > 1), D2H,
    exact inversion -- and returns the histogram (np.uint64) on every rank.  The MOMENTS
    scheme's moment pass runs on a side stream beside the build.  With ``timing=True``
    every step records HIP events (on the streams the work runs on) around the build, the
    count and the all-reduce; ``timings()`` averages them.  bench.py times this object."""

    def __init__(self, codes, code_bits=None, scheme=_lib.SCHEME_AUTO, group=None, device=None):
        import torch
        self.group = group
        self.world, self.rank = _group_info(group)
        # inside an initialised process group the counts are always all-reduced (a one-rank
        # group too: the same collective path as N ranks, a no-op on the values)
        self._reduce = _in_group()
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        if isinstance(codes, np.ndarray):
            host = np.ascontiguousarray(codes, dtype=np.uint64).reshape(-1)
            self.d_codes = torch.from_numpy(host.view(np.int64)).to(self.device)
        else:
            self.d_codes = codes.to(device=self.device, dtype=torch.int64).contiguous().reshape(-1)
            host = None
        n = int(self.d_codes.numel())
        if code_bits is None:
            if host is None:
                host = self.d_codes.cpu().numpy().view(np.uint64)
            code_bits = max(1, int(np.bitwise_or.reduce(host)).bit_length()) if n else 1
        self.n = n
        self.plan = _lib.AllPairsPlan(self.d_codes.data_ptr(), n, code_bits, scheme=scheme)
        self._plan_args = (n, code_bits, scheme)
        self.begin, self.end = item_range(self.plan.items, self.rank, self.world)
        self.counts = torch.zeros(self.plan.ncounts, dtype=torch.int64, device=self.device)
        self.stream = torch.cuda.current_stream(self.device)
        self.side = torch.cuda.Stream(self.device)
        self._ev = {k: torch.cuda.Event(enable_timing=True) for k in
                    ("b0", "b1", "c1", "a1", "m0", "m1")}
        self._ev_zero, self._ev_mom = torch.cuda.Event(), torch.cuda.Event()
        self._t = {"build_ms": [], "count_ms": [], "allreduce_us": [], "moments_ms": []}

    @property
    def scheme(self):
        return self.plan.scheme

    def my_pairs(self):
        return self.plan.range_pairs(self.begin, self.end)

    def step(self, timing=False):
        import torch.distributed as dist
        ev, s, side, sptr = self._ev, self.stream, self.side, self.stream.cuda_stream
        self.counts.zero_()
        moments = self.plan.scheme == _lib.SCHEME_MOMENTS
        if moments:  # independent of the table: beside the build
            self._ev_zero.record(s)
            side.wait_event(self._ev_zero)
            if timing:
                ev["m0"].record(side)
            self.plan.moments(self.counts.data_ptr(), self.rank, self.world, side.cuda_stream)
            if timing:
                ev["m1"].record(side)
            self._ev_mom.record(side)
        if timing:
            ev["b0"].record(s)
        self.plan.build(sptr, self.begin, self.end)  # only what this rank's items read
        if moments:
            s.wait_event(self._ev_mom)
        if timing:
            ev["b1"].record(s)
        self.plan.count(self.counts.data_ptr(), self.begin, self.end, 0, sptr)
        if timing:
            ev["c1"].record(s)
        if self._reduce:
            dist.all_reduce(self.counts, op=dist.ReduceOp.SUM, group=self.group)
        if timing:
            ev["a1"].record(s)
        host = self.counts.cpu().numpy().astype(np.int64).view(np.uint64)  # syncs the stream
        hist = _lib.counts_to_hist(host, self.plan.scheme, self.plan.nbins)
        if timing:
            self._t["build_ms"].append(ev["b0"].elapsed_time(ev["b1"]))
            self._t["count_ms"].append(ev["b1"].elapsed_time(ev["c1"]))
            self._t["allreduce_us"].append(1e3 * ev["c1"].elapsed_time(ev["a1"]))
            if moments:
                self._t["moments_ms"].append(ev["m0"].elapsed_time(ev["m1"]))
        return hist

    #: where run() builds: "side" -- a build stream beside the previous step's count (and the
    #: count buffer zeroed there too), "main" -- in line on the main stream before the count
    build_on = "side"

    def run(self, steps, timing=False):
        """``steps`` whole steps, software-pipelined two deep; returns their histograms.

        Every step does all of ``step()``'s work -- zero, build, count, all-reduce, D2H,
        exact inversion -- with one of two plans and count buffers: step k + 1's build runs
        on a build stream as soon as its plan's count of step k - 1 is done (beside step k's
        count; ``build_on = "main"`` keeps it in line instead) and is enqueued before step k's
        tail, its count is queued on the main stream before the host waits for step k - 1, and
        step k's all-reduce and read-back run on a tail stream, so they and the host's inversion
        overlap the next step's kernels instead of leaving the GPU idle.  The main stream waits
        on one other stream per step at most (a cross-queue wait costs the count ≈10-20 µs of
        idle GPU, rocprof trace)."""
        import torch
        import torch.distributed as dist
        if steps <= 0:
            return []
        if not hasattr(self, "_pipe"):
            dev = self.device
            n, code_bits, _ = self._plan_args
            # the second plan takes the first one's RESOLVED scheme (AUTO resolves by n and the
            # launch-shape knobs, which may have changed since), so both share one geometry
            twin = _lib.AllPairsPlan(self.d_codes.data_ptr(), n, code_bits, scheme=self.plan.scheme)
            if (twin.scheme, twin.items, twin.ncounts, twin.nbins) != \
                    (self.plan.scheme, self.plan.items, self.plan.ncounts, self.plan.nbins):
                twin.close()
                raise RuntimeError("second plan's geometry differs from the first's")
            self._pipe = {
                "plans": [self.plan, twin],
                "build": torch.cuda.Stream(dev),
                "built": [torch.cuda.Event() for _ in range(2)],
                "counts": [self.counts, torch.zeros_like(self.counts)],
                "host": [torch.zeros(self.plan.ncounts, dtype=torch.int64).pin_memory() for _ in range(2)],
                "tail": torch.cuda.Stream(dev),
                # timing events per step, k mod 4 (step k + 1's build and count are enqueued before
                # the host reads step k - 1's), and each plan's count-done event for the waits
                "ev": [{k: torch.cuda.Event(enable_timing=True) for k in ("b0", "b1", "c0", "c1", "a1", "m0", "m1")}
                       for _ in range(4)],
                "cdone": [torch.cuda.Event() for _ in range(2)],
                "done": [torch.cuda.Event() for _ in range(2)],
                "zero": [torch.cuda.Event() for _ in range(2)],
                "mom": [torch.cuda.Event() for _ in range(2)],
            }
        pp = self._pipe
        s, side, tail, sptr = self.stream, self.side, pp["tail"], self.stream.cuda_stream
        moments = self.plan.scheme == _lib.SCHEME_MOMENTS

        side_build = self.build_on == "side" and not moments
        bs = pp["build"] if side_build else s

        def build(k):
            b = k & 1
            counts, ev, plan = pp["counts"][b], pp["ev"][k & 3], pp["plans"][b]
            if side_build:
                bs.wait_event(pp["cdone"][b])  # this plan's count two steps ago no longer reads its tables
                bs.wait_event(pp["done"][b])  # this buffer's read-back two steps ago has finished
                with torch.cuda.stream(bs):
                    counts.zero_()
            if timing:
                ev["b0"].record(bs)
            plan.build(bs.cuda_stream, self.begin, self.end)
            if timing:
                ev["b1"].record(bs)
            if side_build:
                pp["built"][b].record(bs)
            else:
                s.wait_event(pp["done"][b])  # this buffer's read-back two steps ago has finished
                counts.zero_()

        def count(k):
            b = k & 1
            counts, ev, plan = pp["counts"][b], pp["ev"][k & 3], pp["plans"][b]
            if moments:
                pp["zero"][b].record(s)
                side.wait_event(pp["zero"][b])
                if timing:
                    ev["m0"].record(side)
                plan.moments(counts.data_ptr(), self.rank, self.world, side.cuda_stream)
                if timing:
                    ev["m1"].record(side)
                pp["mom"][b].record(side)
                s.wait_event(pp["mom"][b])
            if side_build:
                s.wait_event(pp["built"][b])
            if timing:
                ev["c0"].record(s)
            plan.count(counts.data_ptr(), self.begin, self.end, 0, sptr)
            if timing:
                ev["c1"].record(s)
            pp["cdone"][b].record(s)

        def tail_part(k):
            b = k & 1
            counts, ev = pp["counts"][b], pp["ev"][k & 3]
            tail.wait_event(pp["cdone"][b])
            with torch.cuda.stream(tail):
                if self._reduce:
                    dist.all_reduce(counts, op=dist.ReduceOp.SUM, group=self.group)
                if timing:
                    ev["a1"].record(tail)
                pp["host"][b].copy_(counts, non_blocking=True)
                pp["done"][b].record(tail)

        def finish(k):
            b = k & 1
            pp["done"][b].synchronize()
            host = pp["host"][b].numpy().astype(np.int64).view(np.uint64)
            if timing:
                ev = pp["ev"][k & 3]
                self._t["build_ms"].append(ev["b0"].elapsed_time(ev["b1"]))
                self._t["count_ms"].append(ev["c0"].elapsed_time(ev["c1"]))
                self._t["allreduce_us"].append(1e3 * ev["c1"].elapsed_time(ev["a1"]))
                if moments:
                    self._t["moments_ms"].append(ev["m0"].elapsed_time(ev["m1"]))
            return _lib.counts_to_hist(host, self.plan.scheme, self.plan.nbins)

        hists = []
        if not moments:
            build(0)
            count(0)
        for k in range(steps):
            if moments:  # (the moments pass and its build stay in step order on the main stream)
                build(k)
                count(k)
                tail_part(k)
            else:
                if k + 1 < steps:
                    build(k + 1)
                tail_part(k)
                if k + 1 < steps:
                    count(k + 1)
            if k:
                hists.append(finish(k - 1))
        hists.append(finish(steps - 1))
        return hists

    def reset_timings(self):
        self._t = {k: [] for k in self._t}

    def plans(self):
        """The plan(s) this rank's steps launch on: one for step(), two once run() pipelined."""
        return self._pipe["plans"] if hasattr(self, "_pipe") else [self.plan]

    def kernel_timing(self, mode):
        """Per-launch HIP-event timing of the steps' kernels on the streams they run on
        (sct_allpairs_timing over every plan): mode 1 start, 0 stop, 2 read.  Returns
        {kind: (ms summed, launches)} summed over the plans."""
        tot = {}
        for p in self.plans():
            for k, (ms, n) in p.timing(mode).items():
                a, b = tot.get(k, (0.0, 0))
                tot[k] = (a + ms, b + n)
        return tot

    def timings(self):
        return {k: (float(np.mean(v)) if v else None) for k, v in self._t.items()}

    def close(self):
        if hasattr(self, "_pipe"):
            self._pipe["plans"][1].close()
        self.plan.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def allpairs_histogram_sharded(codes, code_bits=None, group=None, device=None, scheme=_lib.SCHEME_AUTO):
    """Histogram of TwoBit distances over all unordered pairs of `codes` (np.uint64 or a
    torch tensor), sharded over the ranks of `group` (one GPU each).  Call on every rank
    with the same codes; every rank gets the whole histogram."""
    with ShardedAllPairs(codes, code_bits, scheme, group, device) as job:
        return job.step()


def allpairs_wide_sharded(limbs, group=None, device=None):
    """The multi-limb histogram (keys >= 2^64: (n, words) little-endian uint64 limbs, the
    32 * words + 1 bins of ``_lib.hamming_hist_allpairs_wide``) with the tile-pair items
    split into contiguous ranges over the ranks of `group` and one all-reduce of the bins."""
    import torch
    import torch.distributed as dist
    world, rank = _group_info(group)
    limbs = np.ascontiguousarray(limbs, dtype=np.uint64)
    limbs = limbs.reshape(limbs.shape[0], -1) if limbs.ndim else limbs.reshape(0, 1)
    n, words = limbs.shape
    items, nbins = _lib.wide_geometry(n, words)
    b, e = item_range(items, rank, world)
    dev = device or torch.device("cuda", torch.cuda.current_device())
    d = torch.from_numpy(limbs.view(np.int64)).to(dev)
    hist = torch.zeros(nbins, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    _lib.check(_lib.lib().sct_allpairs_wide(d.data_ptr(), n, words, b, e, hist.data_ptr(), nbins, stream))
    if world > 1:
        dist.all_reduce(hist, op=dist.ReduceOp.SUM, group=group)
    return hist.cpu().numpy().view(np.uint64)


def _in_group():
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized()


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


def nearest_sharded(kind, whitelist, queries, max_d=1, code_bits=None, group=None, fn=None, gather=False):
    """Nearest-whitelist correction with the queries split into contiguous ranges, one per
    rank, and the whitelist replicated.  Returns ``(begin, end, index, dist)``: this rank's
    range ``item_range(len(queries), rank, W)`` and its results, with no collective (SURVEY
    8(e): each GPU keeps its own result slice).  Only ``queries[begin:end]`` is read, so
    ``queries`` may be a np.memmap of a file (or any sliceable sequence of uint64 codes).
    ``gather=True`` all-gathers the slices into the whole (index, dist) on every rank
    (then begin, end = 0, len(queries)).  ``fn`` is the per-rank computation (default: the
    GPU path, ``_lib.nearest``)."""
    world, rank = _group_info(group)
    nq = len(queries)
    b, e = item_range(nq, rank, world)
    q = np.ascontiguousarray(queries[b:e], dtype=np.uint64).reshape(-1)
    if code_bits is None:  # the block split's width, as barcode.nearest_whitelist picks it
        wl = np.ascontiguousarray(whitelist, dtype=np.uint64).reshape(-1)
        orv = int(np.bitwise_or.reduce(wl)) if wl.size else 0
        code_bits = min(64, max(orv.bit_length(), kind * (max_d + 1), 1))
    idx, dist_ = (fn or _lib.nearest)(kind, whitelist, q, max_d, code_bits)
    idx, dist_ = np.asarray(idx, dtype=np.int32), np.asarray(dist_, dtype=np.uint8)
    if gather:
        return 0, nq, gather_ranges(idx, nq, group), gather_ranges(dist_, nq, group)
    return b, e, idx, dist_


def encode_sharded(kind, seqs, L, group=None, fn=None, gather=False):
    """TwoBit / ThreeBit batch encode with the records split into contiguous ranges, one per
    rank.  Returns ``(begin, end, *outs)``: this rank's range and what ``fn`` (default
    ``_lib.encode``: codes, gc, flags) returns for ``seqs[begin:end]`` -- the only records
    this rank reads (``seqs`` may be a np.memmap) -- with no collective.  ``gather=True``
    all-gathers every output over the ranks instead."""
    world, rank = _group_info(group)
    nrec = len(seqs)
    b, e = item_range(nrec, rank, world)
    outs = (fn or _lib.encode)(kind, np.asarray(seqs[b:e]), L)
    if gather:
        return (0, nrec) + tuple(gather_ranges(None if o is None else np.asarray(o), nrec, group) for o in outs)
    return (b, e) + tuple(outs)
