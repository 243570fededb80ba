"""GPU, 2 ranks sharing the one GPU of the test box over gloo: the product's per-rank
path (sharding.ShardedAllPairs: plan, build of the rank's items, count of its slice /
item range, all-reduce, inversion) with real kernels on every rank, against the oracle.
The 8-GPU RCCL run itself is the driver's; this proves the per-rank split is exact."""

import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from oracle import oracle as O
from sctools_amd import synthetic

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, seed, scheme, out_path):
    import torch
    import torch.distributed as dist
    from sctools_amd import _lib, sharding
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    _lib.check(_lib.lib().sct_set_device(0))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        codes = synthetic.whitelist_codes(n, 16, seed)
        with sharding.ShardedAllPairs(codes, 32, scheme) as job:
            assert job.scheme == scheme
            assert (job.begin, job.end) == sharding.item_range(job.plan.items, rank, world)
            hist = job.step(timing=True)
            # the pipelined steps bench.py times: three steps, each the whole histogram
            piped = job.run(3, timing=True)
            assert len(piped) == 3 and all(h.tolist() == hist.tolist() for h in piped)
            assert job.timings()["count_ms"] is not None
            mine = job.my_pairs()
        np.savez(out_path % rank, hist=hist.astype(np.int64), mine=mine)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("scheme,world,n", [(2, 2, 20_000), (1, 2, 20_000), (0, 3, 6_000)])
def test_ranks_on_gpu_match_oracle(tmp_path, scheme, world, n):
    out = str(tmp_path / "r%d.npz")
    mp.spawn(_worker, args=(world, _free_port(), n, 41 + scheme, scheme, out), nprocs=world, join=True)
    ref = O.c_hist16(synthetic.whitelist_codes(n, 16, 41 + scheme))[0][:17]
    shares = 0
    for r in range(world):
        z = np.load(out % r)
        assert z["hist"].tolist() == ref.tolist()
        shares += int(z["mine"])
    assert shares == n * (n - 1) // 2


def _worker_737k(rank, world, port, out_path):
    """Config 3's per-rank path at full size: the 737,280-code set, SPECTRAL slice shards,
    two pipelined steps (ShardedAllPairs.run, what bench.py times) and the gloo all-reduce."""
    import torch
    import torch.distributed as dist
    from sctools_amd import _lib, sharding
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    _lib.check(_lib.lib().sct_set_device(0))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n, L, seed = synthetic.CONFIGS[3]
        codes = synthetic.whitelist_codes(n, L, seed)
        with sharding.ShardedAllPairs(codes, 2 * L) as job:
            assert job.scheme == _lib.SCHEME_SPECTRAL
            hists = job.run(2)
            assert hists[0].tolist() == hists[1].tolist()
            np.savez(out_path % rank, hist=hists[0].astype(np.int64), mine=job.my_pairs(),
                     rng=[job.begin, job.end])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_config3_737k_ranks_bin_for_bin(tmp_path, world):
    """Config 3 (BASELINE.json): the 737,280-code all-pairs histogram sharded by transform
    slices over W gloo ranks sharing the box's GPU, every rank's histogram bin for bin
    against the C oracle's count of all 271,790,530,560 pairs (barcode.py:39-46), the ranks'
    slice ranges tiling [0, 2^18) and their pair shares summing to P."""
    out = str(tmp_path / "c3_%d.npz")
    mp.spawn(_worker_737k, args=(world, _free_port(), out), nprocs=world, join=True)
    n, L, seed = synthetic.CONFIGS[3]
    ref = O.c_hist16(synthetic.whitelist_codes(n, L, seed))[0][:17]
    shares, edges = 0, []
    for r in range(world):
        z = np.load(out % r)
        assert z["hist"].tolist() == ref.tolist()
        shares += int(z["mine"])
        edges.append(tuple(z["rng"].tolist()))
    assert shares == n * (n - 1) // 2
    assert edges[0][0] == 0 and edges[-1][1] == 1 << 18
    assert all(a[1] == b[0] for a, b in zip(edges, edges[1:]))


def _records():
    """5,003 random 28-bp ACGT records, (n, 28) uint8."""
    rng = np.random.default_rng(3)
    return np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, (5_003, 28))]


def _wide_limbs():
    """3,001 random 90-bit keys as (n, 2) limbs (the multi-limb path)."""
    rng = np.random.default_rng(8)
    return np.stack([rng.integers(0, 2**63, 3_001, dtype=np.uint64) * np.uint64(2) + np.uint64(1),
                     rng.integers(0, 2**26, 3_001, dtype=np.uint64)], axis=1)


def _worker_records(rank, world, port, out_path):
    """config 4 / config 5 shapes, small: nearest with the queries split over the ranks,
    and the batch encoder with the records split, both through the GPU path on every rank."""
    import torch
    import torch.distributed as dist
    from sctools_amd import _lib, sharding
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    _lib.check(_lib.lib().sct_set_device(0))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        wl3 = synthetic.two_to_three(synthetic.whitelist_codes(20_000, 16, 5), 16)
        q = synthetic.config4_queries(wl3, 30_001, seed=9)[0].cpu().numpy().view(np.uint64)
        qb, qe, idx, dist_ = sharding.nearest_sharded(3, wl3, q, 1)
        eb, ee, codes, gc, flags = sharding.encode_sharded(2, _records(), 28)
        wide = sharding.allpairs_wide_sharded(_wide_limbs())
        np.savez(out_path % rank, qr=[qb, qe], er=[eb, ee], idx=idx, dist=dist_, codes=codes, gc=gc, q=q, wl=wl3,
                 wide=wide)
    finally:
        dist.destroy_process_group()


def test_record_sharding_on_gpu(tmp_path):
    """Contiguous record ranges per rank with no collective: every rank's slice
    equals the oracle's nearest result and encodings on that range; the multi-limb all-pairs
    histogram with its tile-pair items split over the ranks (one all-reduce) equals the oracle's."""
    out = str(tmp_path / "q%d.npz")
    mp.spawn(_worker_records, args=(2, _free_port(), out), nprocs=2, join=True)
    z0 = np.load(out % 0)
    ref_idx, ref_dist = O.c_nearest(3, z0["wl"], z0["q"], 1)
    seqs = [bytes(r) for r in _records()]
    ref_codes = [O.two_bit_encode(s) for s in seqs]
    ref_gc = [s.count(b"C") + s.count(b"G") for s in seqs]
    ends = []
    for r in range(2):
        z = np.load(out % r)
        qb, qe = z["qr"].tolist()
        eb, ee = z["er"].tolist()
        ends.append((qe, ee))
        assert z["idx"].tolist() == ref_idx[qb:qe].tolist()
        assert z["dist"].tolist() == ref_dist[qb:qe].tolist()
        assert z["codes"].reshape(-1).astype(np.uint64).tolist() == ref_codes[eb:ee]
        assert z["gc"].tolist() == ref_gc[eb:ee]
        assert z["wide"].tolist() == O.c_hist_wide(_wide_limbs()).tolist()
    assert ends[-1] == (ref_idx.size, len(seqs))


def _worker_rccl(rank, world, port, out_path):
    """the RCCL stack as bench.py's ranks use it: nccl group bound to the device, an
    all-reduce / all-gather / barrier of CUDA tensors, and ShardedAllPairs inside the group."""
    import torch
    import torch.distributed as dist
    from sctools_amd import _lib, sharding
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    try:
        _lib.check(_lib.lib().sct_set_device(0))
        t = torch.arange(18, dtype=torch.int64, device=dev)
        dist.all_reduce(t)
        rows = [torch.zeros(3, dtype=torch.float64, device=dev) for _ in range(world)]
        dist.all_gather(rows, torch.tensor([rank, 1.5, 2.5], dtype=torch.float64, device=dev))
        dist.barrier()
        codes = synthetic.whitelist_codes(5_000, 16, 3)
        with sharding.ShardedAllPairs(codes, 32, _lib.SCHEME_SPECTRAL) as job:
            hist = job.step(timing=True)
            # bench.py's pipelined steps: the all-reduce from the tail stream over RCCL
            piped = job.run(3, timing=True)
            assert all(h.tolist() == hist.tolist() for h in piped)
            assert job.timings()["allreduce_us"] is not None
        np.savez(out_path % rank, t=t.cpu().numpy(), rows=torch.stack(rows).cpu().numpy(), hist=hist.astype(np.int64),
                 backend=np.array([dist.get_backend()]))
    finally:
        dist.destroy_process_group()


def test_rccl_group_on_gpu(tmp_path):
    """One rank (a box has one GPU; RCCL refuses two ranks on one device): the nccl (= RCCL)
    backend initialises bound to the device and its collectives run, as in bench.py."""
    out = str(tmp_path / "n%d.npz")
    mp.spawn(_worker_rccl, args=(1, _free_port(), out), nprocs=1, join=True)
    z = np.load(out % 0)
    assert z["t"].tolist() == list(range(18))
    assert z["rows"].tolist() == [[0.0, 1.5, 2.5]]
    assert str(z["backend"][0]) == "nccl"
    assert z["hist"].tolist() == O.c_hist16(synthetic.whitelist_codes(5_000, 16, 3))[0][:17].tolist()
