"""Secondary measurements for SURVEY.md §8(d) rows other than the headline
(bench.py): the HBM-bound encoder, nearest-whitelist correction (config 4) and the
3.69M all-pairs (config 5), one GPU.  Prints one JSON object per measurement.

  python tools/bench_paths.py [--reads 1000000000] [--queries 100000000] [--skip-allpairs5]

Encoder (config 5 read stream): reads are random 28-bp ACGT records generated on the
device; one launch of sct_encode(kind=2) writes codes (uint64), GC (uint8) and flags
(uint8).  Algorithmic bytes/read = 28 + 8 + 1 + 1 = 38.
Nearest (config 4): whitelist = the config-2 737,280 codes re-encoded as ThreeBit;
100M queries = 50% exact whitelist draws, 25% one substitution, 15% one N, 10% random,
built on the device from the seeded whitelist.
"""

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from sctools_amd import _lib, synthetic  # noqa: E402

HBM_PEAK = 8.0e12


def timed(fn, reps, stream):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0.record(stream)
        fn()
        e1.record(stream)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts)), float(np.min(ts))


def bench_encode(n_reads, L=28):
    dev = torch.device("cuda")
    s = torch.cuda.current_stream()
    lut = torch.tensor(list(b"ACGT"), dtype=torch.uint8, device=dev)
    g = torch.Generator(device=dev).manual_seed(5)
    seqs = lut[torch.randint(0, 4, (n_reads, L), device=dev, dtype=torch.uint8, generator=g).long()] \
        if n_reads * L <= 2 ** 31 else None
    if seqs is None:  # build in slices to bound the int64 index temporaries
        seqs = torch.empty((n_reads, L), dtype=torch.uint8, device=dev)
        step = 2 ** 26
        for a in range(0, n_reads, step):
            b = min(n_reads, a + step)
            seqs[a:b] = lut[torch.randint(0, 4, (b - a, L), device=dev, generator=g).long()]
    codes = torch.empty(n_reads, dtype=torch.int64, device=dev)
    gc = torch.empty(n_reads, dtype=torch.uint8, device=dev)
    flags = torch.empty(n_reads, dtype=torch.uint8, device=dev)
    lib = _lib.lib()

    def run():
        _lib.check(lib.sct_encode(2, _lib._vp(seqs.data_ptr()), n_reads, L, L, _lib._vp(codes.data_ptr()),
                                  _lib._vp(gc.data_ptr()), _lib._vp(flags.data_ptr()), _lib._vp(s.cuda_stream)))

    med, mn = timed(run, 5, s)
    # spot-check parity of a slice against a host re-encode through the drop-in's batch path
    k = min(4096, n_reads)
    host = seqs[:k].cpu().numpy()
    ref = np.zeros(k, dtype=np.uint64)
    for p in range(L):
        ch = host[:, p]
        val = np.select([ch == 65, ch == 67, ch == 84, ch == 71], [0, 1, 2, 3]).astype(np.uint64)
        ref = (ref << np.uint64(2)) | val
    assert np.array_equal(codes[:k].cpu().numpy().view(np.uint64), ref), "encode parity"
    byts = n_reads * (L + 8 + 1 + 1)
    del seqs, codes, gc, flags
    torch.cuda.empty_cache()
    return {"path": "encode TwoBit+GC (config 5 read stream)", "reads": n_reads, "L": L,
            "median_ms": med, "min_ms": mn, "reads_per_s": n_reads / (med * 1e-3),
            "roofline": {"bound": "hbm", "achieved": byts / (med * 1e-3) / 1e9, "peak": HBM_PEAK / 1e9,
                         "unit": "GB/s", "frac": byts / (med * 1e-3) / HBM_PEAK,
                         "bytes_per_read": L + 10}}


def bench_encode_stream(n_reads, L=28):
    """Host-resident reads (pinned by the caller, as a streaming reader would): the
    PCIe-inclusive rate of sct_encode_stream_host."""
    dev = torch.device("cuda")
    lut = torch.tensor(list(b"ACGT"), dtype=torch.uint8, device=dev)
    g = torch.Generator(device=dev).manual_seed(6)
    host = torch.empty((n_reads, L), dtype=torch.uint8, pin_memory=True)
    step = 2 ** 25
    for a in range(0, n_reads, step):
        b = min(n_reads, a + step)
        host[a:b] = lut[torch.randint(0, 4, (b - a, L), device=dev, generator=g).long()].cpu()
    codes = torch.empty(n_reads, dtype=torch.int64, pin_memory=True)
    gc = torch.empty(n_reads, dtype=torch.uint8, pin_memory=True)
    flags = torch.empty(n_reads, dtype=torch.uint8, pin_memory=True)
    lib = _lib.lib()
    ts = []
    for _ in range(3):
        t = time.perf_counter()
        _lib.check(lib.sct_encode_stream_host(2, _lib._vp(host.data_ptr()), n_reads, L, _lib._vp(codes.data_ptr()),
                                              _lib._vp(gc.data_ptr()), _lib._vp(flags.data_ptr()), 1 << 24))
        ts.append(time.perf_counter() - t)
    sec = float(np.median(ts))
    k = 1000
    ref = np.zeros(k, dtype=np.uint64)
    hv = host[:k].numpy()
    for p in range(L):
        ch = hv[:, p]
        ref = (ref << np.uint64(2)) | np.select([ch == 65, ch == 67, ch == 84, ch == 71], [0, 1, 2, 3]).astype(np.uint64)
    assert np.array_equal(codes[:k].numpy().view(np.uint64), ref), "stream encode parity"
    return {"path": "encode TwoBit+GC host-resident stream (PCIe-inclusive, config 5)", "reads": n_reads,
            "L": L, "median_s": sec, "reads_per_s": n_reads / sec,
            "pcie_bytes_per_s": n_reads * (L + 10) / sec,
            "note": "H2D L bytes + D2H 10 bytes per read over PCIe Gen5 x16 (63 GB/s spec per direction)"}


def bench_nearest(nq, max_d=1):
    dev = torch.device("cuda")
    s = torch.cuda.current_stream()
    n, L, seed = synthetic.CONFIGS[2]
    wl = synthetic.two_to_three(synthetic.whitelist_codes(n, L, seed), L)
    d_wl = torch.from_numpy(wl.view(np.int64)).to(dev)
    q, _, _ = synthetic.config4_queries(wl, nq, seed=4, device=dev)
    g = torch.Generator(device=dev).manual_seed(4)
    idx = torch.empty(nq, dtype=torch.int32, device=dev)
    dist = torch.empty(nq, dtype=torch.uint8, device=dev)
    t0 = time.perf_counter()
    plan = _lib.NearestPlan(3, d_wl.data_ptr(), n, 3 * L, max_d, s.cuda_stream)
    torch.cuda.synchronize()
    cold_ms = (time.perf_counter() - t0) * 1e3  # includes first-use module loads
    plan.close()
    t0 = time.perf_counter()
    plan = _lib.NearestPlan(3, d_wl.data_ptr(), n, 3 * L, max_d, s.cuda_stream)
    torch.cuda.synchronize()
    build_ms = (time.perf_counter() - t0) * 1e3  # allocation + bucketing, warm

    def run():
        plan.query(q.data_ptr(), nq, idx.data_ptr(), dist.data_ptr(), s.cuda_stream)

    med, mn = timed(run, 5, s)
    # parity spot check against the oracle brute force on a sample
    from oracle import oracle as O
    samp = torch.randint(0, nq, (2000,), device=dev, generator=g)
    ridx, rdist = O.c_nearest(3, wl, q[samp].cpu().numpy().view(np.uint64), max_d)
    assert np.array_equal(idx[samp].cpu().numpy(), ridx) and np.array_equal(dist[samp].cpu().numpy(), rdist)
    hist = torch.bincount(idx.clamp(min=-2).add(2).clamp(max=2).long(), minlength=3).tolist()
    plan.close()
    byts = nq * (8 + 4 + 1)
    return {"path": "nearest whitelist ThreeBit max_d=%d (config 4)" % max_d, "whitelist": n, "queries": nq,
            "median_ms": med, "min_ms": mn, "queries_per_s": nq / (med * 1e-3), "index_build_ms": build_ms, "index_build_cold_ms": cold_ms,
            "brute_force_equiv_pairs_per_s": nq * n / (med * 1e-3),
            "outcome_counts": {"tie": hist[0], "none": hist[1], "hit": hist[2]},
            "roofline": {"bound": "hbm", "achieved": byts / (med * 1e-3) / 1e9, "peak": HBM_PEAK / 1e9,
                         "unit": "GB/s", "frac": byts / (med * 1e-3) / HBM_PEAK, "bytes_per_query": 13,
                         "note": "stream bytes only; bucket reads are L2/MALL-resident"}}


def bench_fastq(n_rec):
    """Device-resident synthetic R1 FASTQ (69-byte records: 12-char name, 26-bp read, '+',
    26 qualities): index (lines -> records, name check), slice CB 0:16 and UMI 16:24
    sequences and qualities (TenXV2), TwoBit-encode the CBs with GC."""
    dev = torch.device("cuda")
    s = torch.cuda.current_stream()
    g = torch.Generator(device=dev).manual_seed(6)
    acgt = torch.tensor(list(b"ACGT"), dtype=torch.uint8, device=dev)
    rec = torch.empty((n_rec, 69), dtype=torch.uint8, device=dev)
    rec[:, 0] = ord("@")
    rec[:, 1:12] = ord("r")
    rec[:, 12] = 10
    rec[:, 13:39] = acgt[torch.randint(0, 4, (n_rec, 26), device=dev, generator=g)]
    rec[:, 39] = 10
    rec[:, 40] = ord("+")
    rec[:, 41] = 10
    rec[:, 42:68] = ord("F")
    rec[:, 68] = 10
    buf = rec.reshape(-1)
    nbytes = buf.numel()
    seqs = torch.empty(n_rec * 24, dtype=torch.uint8, device=dev)  # span-major: CB rows, UMI rows
    quals = torch.empty_like(seqs)
    cb = seqs[:n_rec * 16].view(n_rec, 16)
    umi = seqs[n_rec * 16:].view(n_rec, 8)
    codes = torch.empty(n_rec, dtype=torch.int64, device=dev)
    gc = torch.empty(n_rec, dtype=torch.uint8, device=dev)
    flags = torch.empty(n_rec, dtype=torch.uint8, device=dev)
    L = _lib.lib()
    box = {}

    def run():
        ix = _lib.FastqIndex(buf.data_ptr(), nbytes, [nbytes], False, s.cuda_stream)
        ix.extract_spans(buf.data_ptr(), [(0, 16), (16, 24)], seqs.data_ptr(), quals.data_ptr(),
                         stream=s.cuda_stream)
        _lib.check(L.sct_encode(2, _lib._vp(cb.data_ptr()), n_rec, 16, 16, _lib._vp(codes.data_ptr()),
                                _lib._vp(gc.data_ptr()), _lib._vp(flags.data_ptr()), _lib._vp(s.cuda_stream)))
        box["n"] = ix.nrecords
        ix.close()

    med, mn = timed(run, 5, s)
    assert box["n"] == n_rec
    # parity spot check: CB rows equal the read bytes, codes equal the oracle TwoBit encode
    from oracle import oracle as O
    i = torch.randint(0, n_rec, (64,), device=dev, generator=g)
    assert torch.equal(cb[i], rec[i, 13:29]) and torch.equal(umi[i], rec[i, 29:37])
    host = cb[i].cpu().numpy()
    assert [O.two_bit_encode(bytes(r)) for r in host] == [int(x) for x in codes[i].cpu().numpy().view(np.uint64)]
    byts = nbytes + n_rec * (16 + 8) * 2 + n_rec * 10  # FASTQ read + slices written + codes/gc/flags
    return {"path": "FASTQ R1 CB/UMI extraction + TwoBit encode (device-resident)", "records": n_rec,
            "fastq_bytes": nbytes, "median_ms": med, "min_ms": mn, "records_per_s": n_rec / (med * 1e-3),
            "fastq_GB_per_s": nbytes / (med * 1e-3) / 1e9,
            "roofline": {"bound": "hbm", "achieved": byts / (med * 1e-3) / 1e9, "peak": HBM_PEAK / 1e9,
                         "unit": "GB/s", "frac": byts / (med * 1e-3) / HBM_PEAK,
                         "note": "algorithmic bytes: the FASTQ once + slices + codes; the index "
                                 "reads the buffer twice (count, write) and syncs once for its size"}}


def bench_allpairs5():
    dev = torch.device("cuda")
    s = torch.cuda.current_stream()
    n, L, seed = synthetic.CONFIGS[5]
    codes = synthetic.whitelist_codes(n, L, seed)
    d = torch.from_numpy(codes.view(np.int64)).to(dev)
    plan = _lib.AllPairsPlan(d.data_ptr(), n, 2 * L)
    counts = torch.zeros(plan.ncounts, dtype=torch.int64, device=dev)

    def run():
        counts.zero_()
        plan.build(s.cuda_stream)
        plan.moments(counts.data_ptr(), stream=s.cuda_stream)
        plan.count(counts.data_ptr(), stream=s.cuda_stream)

    med, mn = timed(run, 3, s)
    hist = plan.counts_to_hist(counts.cpu().numpy().view(np.uint64))
    assert int(hist.sum()) == plan.pairs
    plan.close()
    return {"path": "all-pairs histogram config 5 (3,686,400 codes)", "pairs": plan.pairs, "median_ms": med,
            "min_ms": mn, "pairs_per_s": plan.pairs / (med * 1e-3), "hist": [int(x) for x in hist]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=1_000_000_000)
    ap.add_argument("--queries", type=int, default=100_000_000)
    ap.add_argument("--skip-allpairs5", action="store_true")
    ap.add_argument("--fastq-records", type=int, default=20_000_000)
    ap.add_argument("--stream-reads", type=int, default=250_000_000)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    _lib.check(_lib.lib().sct_set_device(0))
    if a.reads:
        print(json.dumps(bench_encode(a.reads)), flush=True)
    if a.stream_reads:
        print(json.dumps(bench_encode_stream(a.stream_reads)), flush=True)
    if a.queries:
        print(json.dumps(bench_nearest(a.queries, 1)), flush=True)
    if a.fastq_records:
        print(json.dumps(bench_fastq(a.fastq_records)), flush=True)
    if not a.skip_allpairs5:
        print(json.dumps(bench_allpairs5()), flush=True)


if __name__ == "__main__":
    main()
