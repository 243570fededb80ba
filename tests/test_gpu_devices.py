"""The library's in-process device split (devices.cpp, include/sctools_hip.h "several devices"),
the one-shot calls' device-memory policy, and the plan destroy contract.

The box has one GPU, so the device lists repeat ordinal 0: every slot is then a logical shard on
its own worker thread, own host stage and own plan, exactly as on a node with distinct GPUs; only
the RCCL-free host sum of the counts is the same either way.  Every result is checked bin for bin
(all-pairs) or element for element (nearest, encode) against the C oracle or the one-device call.
"""

import numpy as np
import pytest

from oracle import oracle as O
from sctools_amd import _lib, barcode, encodings, synthetic

pytestmark = pytest.mark.gpu

_REF = {}


def _ref16(key, codes):
    if key not in _REF:
        _REF[key] = O.c_hist16(codes)[0][:17].tolist()
    return _REF[key]


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0, 0], [0, 0, 0]])
def test_allpairs_737k_devices_bin_for_bin(devices):
    """Config 2 (737,280 codes, SPECTRAL) split over 2, 3 and 4 device slots: each slot counts its
    slice range on its own replica; the summed counts invert to the oracle's histogram of all
    271,790,530,560 pairs, and the drop-in summary over those devices equals the oracle's."""
    n, L, seed = synthetic.CONFIGS[2]
    codes = synthetic.whitelist_codes(n, L, seed)
    ref = _ref16("c2", codes)
    hist = _lib.hamming_hist_allpairs(codes, 32, distinct=True, devices=devices)
    assert hist.astype(np.int64).tolist() == ref
    prev = _lib.get_devices()
    _lib.set_devices(devices)
    try:
        s = barcode.Barcodes({int(c): 1 for c in codes}, 16)
        assert s.summarize_hamming_distances() == O.summary_from_hist_numpy(ref)
    finally:
        _lib.set_devices(None if prev == [0] else prev)


def test_allpairs_config5_devices_bin_for_bin():
    """Config 5 (3,686,400 codes, 16-bit columns) over 4 slots vs the oracle's 6.79e12 pairs."""
    n, L, seed = synthetic.CONFIGS[5]
    codes = synthetic.whitelist_codes(n, L, seed)
    hist = _lib.hamming_hist_allpairs(codes, 32, distinct=True, devices=[0, 0, 0, 0])
    assert hist.astype(np.int64).tolist() == _ref16("c5", codes)


@pytest.mark.parametrize("n", [0, 1, 2, 3, 5000, 40_000])
def test_allpairs_devices_small_and_pair_schemes(n):
    """Below the SPECTRAL threshold (MOMENTS / SUBSETS pair kernels: item ranges and moment parts
    per slot) and the degenerate sizes, over 3 slots; 12-bit codes take SUBSETS."""
    codes = synthetic.whitelist_codes(max(n, 1), 16, seed=n + 3)[:n]
    got = _lib.hamming_hist_allpairs(codes, 32, devices=[0, 0, 0])
    assert got.astype(np.int64).tolist() == O.c_hist_rows(codes)[:17].tolist()
    small = (codes & np.uint64(0xFFF))
    got12 = _lib.hamming_hist_allpairs(small, 12, devices=[0, 0, 0])
    assert got12.astype(np.int64).tolist() == O.c_hist_rows(small)[:7].tolist()


def test_devices_errors():
    codes = synthetic.whitelist_codes(1000, 16, seed=1)
    with pytest.raises(ValueError, match="device"):
        _lib.hamming_hist_allpairs(codes, 32, devices=[0, 99])
    with pytest.raises(ValueError):
        _lib.set_devices([])


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_nearest_devices(devices):
    """Nearest-whitelist over several slots (contiguous query ranges, the index on every slot):
    the one-device result, and the brute force on a sample; WhitelistCorrector the same, batch
    after batch."""
    torch = pytest.importorskip("torch")
    n, L, seed = synthetic.CONFIGS[4]
    wl = synthetic.two_to_three(synthetic.whitelist_codes(n, L, seed), L)
    q, _, _ = synthetic.config4_queries(wl, 5_000_003, seed=9, device="cuda")
    q = q.cpu().numpy().view(np.uint64)
    i1, d1 = barcode.nearest_whitelist(q, wl, 1, devices=[0])
    im, dm = barcode.nearest_whitelist(q, wl, 1, devices=devices)
    assert np.array_equal(i1, im) and np.array_equal(d1, dm)
    samp = np.random.default_rng(3).integers(0, q.size, 5000)
    ridx, rdist = O.c_nearest(3, wl, q[samp], 1)
    assert np.array_equal(im[samp], ridx) and np.array_equal(dm[samp], rdist)
    corr = barcode.WhitelistCorrector(wl, 1, devices=devices)
    try:
        for a, b in ((0, 7), (7, 7), (7, 1_000_000), (1_000_000, q.size)):
            ic, dc = corr.nearest(q[a:b])
            assert np.array_equal(ic, i1[a:b]) and np.array_equal(dc, d1[a:b])
    finally:
        corr.close()
    del torch


def test_encode_stream_devices():
    """The host encode stream over 3 slots: the one-device codes, GC and flags."""
    rng = np.random.default_rng(71)
    n, L = 4_500_011, 28
    seqs = np.frombuffer(b"ACGTacgtN", np.uint8)[rng.integers(0, 9, (n, L))]
    one = _lib.encode_stream(2, seqs, devices=[0])
    many = _lib.encode_stream(2, seqs, devices=[0, 0, 0])
    for a, b in zip(one, many):
        assert np.array_equal(a, b)
    for r in range(0, n, 499_999):
        s = seqs[r].tobytes()
        if b"N" not in s:
            assert int(many[0][r]) == O.two_bit_encode(s)


def test_one_shot_call_leaves_no_device_memory():
    """by default a one-shot summary frees every device buffer it mapped
    (mem_get_info back to the free bytes before the call); keep_workspace(True) keeps the
    workspace for the next call, release_device_memory() hands it back."""
    torch = pytest.importorskip("torch")
    import sctools_amd
    n, L, seed = synthetic.CONFIGS[2]
    codes = synthetic.whitelist_codes(n, L, seed)
    b = barcode.Barcodes({int(c): 1 for c in codes}, 16)
    ref = O.summary_from_hist_numpy(_ref16("c2", codes))
    prev = sctools_amd.keep_workspace(False)
    try:
        sctools_amd.release_device_memory()
        assert b.summarize_hamming_distances() == ref  # (first call: code objects, host stage)
        torch.cuda.synchronize()
        free0 = torch.cuda.mem_get_info()[0]
        assert b.summarize_hamming_distances() == ref
        torch.cuda.synchronize()
        assert torch.cuda.mem_get_info()[0] == free0
        sctools_amd.keep_workspace(True)
        assert b.summarize_hamming_distances() == ref
        kept = free0 - torch.cuda.mem_get_info()[0]
        assert kept >= 4 << 30  # the transform intermediate stays mapped
        assert b.summarize_hamming_distances() == ref
        assert free0 - torch.cuda.mem_get_info()[0] == kept  # (reused: nothing new mapped)
        sctools_amd.release_device_memory()
        torch.cuda.synchronize()
        assert torch.cuda.mem_get_info()[0] >= free0
    finally:
        sctools_amd.keep_workspace(prev)


def test_plan_destroy_waits_for_enqueued_work():
    """a plan destroyed right after work was enqueued on a side stream returns
    only once that work has completed (the event recorded after it has passed when destroy
    returns, with no synchronisation by the caller), and the results are exact."""
    torch = pytest.importorskip("torch")
    side = torch.cuda.Stream()
    # all-pairs: 737K SPECTRAL count
    n, L, seed = synthetic.CONFIGS[2]
    codes = synthetic.whitelist_codes(n, L, seed)
    d = torch.from_numpy(codes.view(np.int64)).cuda()
    plan = _lib.AllPairsPlan(d.data_ptr(), n, 32, distinct=True)
    counts = torch.zeros(plan.ncounts, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    plan.build(side.cuda_stream)
    plan.count(counts.data_ptr(), stream=side.cuda_stream)
    ev = torch.cuda.Event()
    ev.record(side)
    plan.close()
    assert ev.query(), "all-pairs destroy returned before its enqueued count finished"
    hist = _lib.counts_to_hist(counts.cpu().numpy().view(np.uint64), _lib.SCHEME_SPECTRAL, 17)
    assert hist.astype(np.int64).tolist() == _ref16("c2", codes)
    # nearest: a 20M-query pass on the side stream, the plan destroyed at once
    wl = synthetic.two_to_three(codes, L)
    q, pick, cls = synthetic.config4_queries(wl, 20_000_000, seed=5, device="cuda")
    d_wl = torch.from_numpy(wl.view(np.int64)).cuda()
    idx = torch.empty(q.numel(), dtype=torch.int32, device="cuda")
    dist = torch.empty(q.numel(), dtype=torch.uint8, device="cuda")
    nplan = _lib.NearestPlan(3, d_wl.data_ptr(), wl.size, 48, 1)
    torch.cuda.synchronize()
    nplan.query(q.data_ptr(), q.numel(), idx.data_ptr(), dist.data_ptr(), stream=side.cuda_stream)
    ev2 = torch.cuda.Event()
    ev2.record(side)
    nplan.close()
    assert ev2.query(), "nearest destroy returned before its enqueued query finished"
    exact = cls == 0
    assert torch.equal(idx[exact].long(), pick[exact])
    samp = np.random.default_rng(8).integers(0, q.numel(), 5000)
    ridx, rdist = O.c_nearest(3, wl, q.cpu().numpy().view(np.uint64)[samp], 1)
    assert np.array_equal(idx.cpu().numpy()[samp], ridx) and np.array_equal(dist.cpu().numpy()[samp], rdist)


@pytest.mark.parametrize("pinned_inputs", [True, False])
def test_batch_arrays_streamed(pinned_inputs):
    """Element-wise batch calls above the stream threshold (8 MB) run chunked over the pipeline
    streams (host_items): hamming_distance_array (both kinds), decode_array, gc_content_array on
    3,000,017 items from page-locked or pageable inputs equal the same calls made in small pieces
    (one staged round trip each) and the numpy formulas on a sample."""
    rng = np.random.default_rng(17 + pinned_inputs)
    n = 3_000_017
    a = rng.integers(0, 1 << 32, n, dtype=np.uint64)
    b = a ^ (rng.integers(0, 1 << 32, n, dtype=np.uint64) & np.uint64(0x00F0000F))
    if pinned_inputs:
        pa, pb = _lib.pinned.empty(n, np.uint64), _lib.pinned.empty(n, np.uint64)
        pa[:], pb[:] = a, b
        assert _lib.host_pinned(pa) and _lib.host_pinned(pb)
        a, b = pa, pb
    T2, T3, t16 = encodings.TwoBit, encodings.ThreeBit, encodings.TwoBit(16)
    full = [T2.hamming_distance_array(a, b), T3.hamming_distance_array(a, b), t16.decode_array(a),
            t16.gc_content_array(a)]
    step = 200_000  # pieces of 2.4-4.8 MB: below the threshold
    pieces = [np.concatenate([f(a[i:i + step], b[i:i + step]) for i in range(0, n, step)])
              for f in (T2.hamming_distance_array, T3.hamming_distance_array, lambda x, y: t16.decode_array(x),
                        lambda x, y: t16.gc_content_array(x))]
    for f, p in zip(full, pieces):
        assert np.array_equal(f, p)
    s = rng.integers(0, n, 20_000)
    x = a[s] ^ b[s]
    w2 = [bin(int(v)).count("1") for v in (x | (x >> np.uint64(1))) & np.uint64(0x5555555555555555)]
    assert full[0][s].tolist() == w2
    assert full[3][s].tolist() == [bin(int(v) & 0x55555555).count("1") for v in a[s]]
    assert [bytes(v) for v in full[2][s[:500]]] == [O.two_bit_decode(int(v), 16) for v in a[s[:500]]]
