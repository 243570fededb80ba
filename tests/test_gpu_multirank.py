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
        idx, dist_ = sharding.nearest_sharded(3, wl3, q, 1)
        codes, gc, flags = sharding.encode_sharded(2, _records(), 28)
        wide = sharding.allpairs_wide_sharded(_wide_limbs())
        np.savez(out_path % rank, idx=idx, dist=dist_, codes=codes, gc=gc, q=q, wl=wl3, wide=wide)
    finally:
        dist.destroy_process_group()


def test_record_sharding_on_gpu(tmp_path):
    """Contiguous record ranges per rank (no reduction, one all-gather): every rank ends with
    the oracle's whole nearest result and the oracle's encodings; the multi-limb all-pairs
    histogram with its tile-pair items split over the ranks equals the oracle's."""
    out = str(tmp_path / "q%d.npz")
    mp.spawn(_worker_records, args=(2, _free_port(), out), nprocs=2, join=True)
    z0 = np.load(out % 0)
    ref_idx, ref_dist = O.c_nearest(3, z0["wl"], z0["q"], 1)
    seqs = [bytes(r) for r in _records()]
    ref_codes = [O.two_bit_encode(s) for s in seqs]
    for r in range(2):
        z = np.load(out % r)
        assert z["idx"].tolist() == ref_idx.tolist()
        assert z["dist"].tolist() == ref_dist.tolist()
        assert z["codes"].reshape(-1).astype(np.uint64).tolist() == ref_codes
        assert z["gc"].tolist() == [s.count(b"C") + s.count(b"G") for s in seqs]
        assert z["wide"].tolist() == O.c_hist_wide(_wide_limbs()).tolist()


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
