"""CPU, world_size 2 (gloo): the multi-GPU orchestration — item partition, count
all-reduce, inversion — without a GPU.  Each rank's per-shard subset counts come from
the C oracle's independent enumeration of the same work items (test-only stand-in
for the kernel, which has its own GPU parity tests); the product code under test is
sctools_amd.sharding.item_range / combine_counts and the library's geometry and
Moebius inversion."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle as O
from sctools_amd import _lib, sharding, synthetic


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _shard_counts(codes, geo, b, e):
    hist = np.zeros(65, dtype=np.int64)
    pairs = np.zeros(1, dtype=np.int64)
    O.c_oracle().oracle_hist_items(codes.ctypes.data, codes.size, geo["rows_per_item"],
                                   geo["cols_per_item"], hist.ctypes.data, b, e, pairs.ctypes.data, 1)
    nb = geo["nbins"]
    counts = np.zeros(nb, dtype=np.int64)
    for m in range(nb):
        counts[m] = sum(int(hist[d]) for d in range(nb) if (d & m) == m)
    assert counts[0] == pairs[0]
    return counts


def _shard_moment_counts(codes, geo, b, e, rank):
    """MOMENTS-scheme counts of one rank: the 13 products of its item range, plus (rank 0
    here; the kernel splits them by position triple) the whole job's agreement moments."""
    hist = np.zeros(65, dtype=np.int64)
    pairs = np.zeros(1, dtype=np.int64)
    O.c_oracle().oracle_hist_items(codes.ctypes.data, codes.size, geo["rows_per_item"],
                                   geo["cols_per_item"], hist.ctypes.data, b, e, pairs.ctypes.data, 1)
    c = O.moment_counts_from_hist(hist[:17]).astype(np.int64)
    c[14:] = O.moments_from_marginals(codes) if rank == 0 else 0
    return c


def _worker_moments(rank, world, port, n, seed, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        codes = synthetic.whitelist_codes(n, 16, seed)
        geo = _lib.allpairs_geometry(n, 32)  # AUTO = MOMENTS at 16 bases: 512-code chunks
        assert geo["cols_per_item"] == 512
        b, e = sharding.item_range(geo["items"], rank, world)
        counts = torch.from_numpy(_shard_moment_counts(codes, geo, b, e, rank))
        hist = sharding.combine_counts(counts, None, _lib.SCHEME_MOMENTS, 17)
        np.save(out_path % rank, hist.astype(np.int64))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 1800)])
def test_sharded_moments_histogram_matches_oracle(tmp_path, world, n):
    port = _free_port()
    out = str(tmp_path / "mhist_%d.npy")
    mp.spawn(_worker_moments, args=(world, port, n, 23, out), nprocs=world, join=True)
    ref = O.c_hist_rows(synthetic.whitelist_codes(n, 16, 23))[:17]
    for r in range(world):
        assert np.load(out % r).tolist() == ref.tolist()


def _worker(rank, world, port, n, seed, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        codes = synthetic.whitelist_codes(n, 16, seed)
        geo = _lib.allpairs_geometry(n, 32)
        b, e = sharding.item_range(geo["items"], rank, world)
        counts = torch.from_numpy(_shard_counts(codes, geo, b, e))
        hist = sharding.combine_counts(counts)
        np.save(out_path % rank, hist.astype(np.int64))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 2500), (3, 1300)])
def test_sharded_histogram_matches_oracle(tmp_path, world, n):
    port = _free_port()
    out = str(tmp_path / "hist_%d.npy")
    mp.spawn(_worker, args=(world, port, n, 17, out), nprocs=world, join=True)
    codes = synthetic.whitelist_codes(n, 16, 17)
    ref = O.c_hist_rows(codes)[:17]
    for r in range(world):
        assert np.load(out % r).tolist() == ref.tolist()


def test_item_range_partitions():
    for items in (0, 1, 7, 1038240):
        for world in (1, 2, 3, 4, 8):
            ranges = [sharding.item_range(items, r, world) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == items
            assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
            sizes = [e - b for b, e in ranges]
            assert max(sizes) - min(sizes) <= 1


def test_geometry_item_count_matches_oracle_enumeration():
    # 737K codes resolve to SPECTRAL (2^18 slice items); the pair-item geometry is MOMENTS'
    assert _lib.allpairs_geometry(737_280, 32)["items"] == 1 << 18
    with _lib.tuning(spectral_min_n=1 << 40):  # AUTO never takes SPECTRAL
        for n in (2, 100, 1024, 1025, 5000, 737_280):
            geo = _lib.allpairs_geometry(n, 32)
            rb, cb = geo["rows_per_item"], geo["cols_per_item"]
            nch = -(-n // cb)
            items = sum(max(0, -(-(min((c + 1) * cb, n) - 1) // rb)) for c in range(nch))
            assert geo["items"] == items
    assert _lib.tune_get("spectral_min_n") == -1


def _worker_spectral(rank, world, port, n, seed, out_path):
    """SPECTRAL counts of one rank: its share of every S_w (the slices it would count;
    here an arbitrary integer split of the oracle's S), n on the rank holding item 0."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        codes = synthetic.whitelist_codes(n, 16, seed)
        full = O.spectral_counts_from_hist(O.c_hist_rows(codes)[:17], n).astype(object)
        share = [int(x) * (rank + 1) // world - int(x) * rank // world for x in full[2:]]
        b, _ = sharding.item_range(1 << 18, rank, world)
        counts = torch.tensor([n if b == 0 else 0, int(full[1]) if b == 0 else 0] + share, dtype=torch.int64)
        hist = sharding.combine_counts(counts, None, _lib.SCHEME_SPECTRAL, 17)
        np.save(out_path % rank, hist.astype(np.int64))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 1500), (3, 700)])
def test_sharded_spectral_histogram_matches_oracle(tmp_path, world, n):
    port = _free_port()
    out = str(tmp_path / "shist_%d.npy")
    mp.spawn(_worker_spectral, args=(world, port, n, 29, out), nprocs=world, join=True)
    ref = O.c_hist_rows(synthetic.whitelist_codes(n, 16, 29))[:17]
    for r in range(world):
        assert np.load(out % r).tolist() == ref.tolist()


def _oracle_nearest(kind, whitelist, queries, max_d, code_bits):
    """Test-only stand-in for the GPU nearest path on this rank's slice."""
    idx, dist_ = O.nearest_bruteforce(kind, [int(x) for x in whitelist], [int(x) for x in queries], max_d)
    return np.asarray(idx, dtype=np.int32), np.asarray(dist_, dtype=np.uint8)


def _oracle_encode(kind, seqs, L):
    enc = O.two_bit_encode if kind == 2 else O.three_bit_encode
    gcf = O.two_bit_gc if kind == 2 else O.three_bit_gc
    codes = np.array([[enc(bytes(r))] for r in seqs], dtype=np.uint64).reshape(-1, 1)
    gc = np.array([gcf(int(c[0]), L) if kind == 2 else gcf(int(c[0])) for c in codes], dtype=np.uint8)
    return codes, gc, np.zeros(len(seqs), dtype=np.uint8)


def _worker_ranges(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(5)
        wl = np.unique(rng.integers(0, 1 << 48, 300, dtype=np.uint64))[:250]
        q = np.concatenate([wl[:40], wl[40:80] ^ np.uint64(1 << 7), rng.integers(0, 1 << 48, 37, dtype=np.uint64)])
        seqs = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=(101, 16))
        # default: this rank's slice only, no collective
        qb, qe, idx, d = sharding.nearest_sharded(3, wl, q, 1, 48, fn=_oracle_nearest)
        eb, ee, codes, gc, flags = sharding.encode_sharded(2, seqs, 16, fn=_oracle_encode)
        # opt-in: the whole result on every rank
        gb, ge, gidx, gd = sharding.nearest_sharded(3, wl, q, 1, 48, fn=_oracle_nearest, gather=True)
        _, _, gcodes, ggc, gflags = sharding.encode_sharded(2, seqs, 16, fn=_oracle_encode, gather=True)
        np.savez(out_path % rank, qr=[qb, qe, gb, ge], er=[eb, ee], idx=idx, d=d, codes=codes, gc=gc, flags=flags,
                 gidx=gidx, gd=gd, gcodes=gcodes, ggc=ggc, gflags=gflags)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_contiguous_range_sharding(tmp_path, world):
    """Config 4 / encoder sharding: contiguous record ranges per rank, each rank
    keeping only its own result slice (no collective); the slices tile the unsharded result.
    The opt-in gather gives every rank the whole result."""
    port = _free_port()
    out = str(tmp_path / "ranges_%d.npz")
    mp.spawn(_worker_ranges, args=(world, port, out), nprocs=world, join=True)
    rng = np.random.default_rng(5)
    wl = np.unique(rng.integers(0, 1 << 48, 300, dtype=np.uint64))[:250]
    q = np.concatenate([wl[:40], wl[40:80] ^ np.uint64(1 << 7), rng.integers(0, 1 << 48, 37, dtype=np.uint64)])
    ridx, rd = _oracle_nearest(3, wl, q, 1, 48)
    seqs = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=(101, 16))
    rcodes, rgc, _ = _oracle_encode(2, seqs, 16)
    assert (ridx[:40] == np.arange(40)).all() and (ridx[40:80] == np.arange(40, 80)).all()
    parts = [np.load(out % r) for r in range(world)]
    for r, z in enumerate(parts):
        qb, qe, gb, ge = z["qr"].tolist()
        eb, ee = z["er"].tolist()
        assert (qb, qe) == sharding.item_range(q.size, r, world) and (gb, ge) == (0, q.size)
        assert (eb, ee) == sharding.item_range(101, r, world)
        assert z["idx"].tolist() == ridx[qb:qe].tolist() and z["d"].tolist() == rd[qb:qe].tolist()
        assert z["codes"].tolist() == rcodes[eb:ee].tolist() and z["gc"].tolist() == rgc[eb:ee].tolist()
        assert z["gidx"].tolist() == ridx.tolist() and z["gd"].tolist() == rd.tolist()
        assert z["gcodes"].shape == (101, 1) and z["gcodes"].tolist() == rcodes.tolist()
        assert z["ggc"].tolist() == rgc.tolist() and z["gflags"].shape == (101,)
    assert np.concatenate([z["idx"] for z in parts]).tolist() == ridx.tolist()
