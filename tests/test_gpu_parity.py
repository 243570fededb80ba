"""GPU parity: the HIP path (through the C ABI / Python drop-in) against the golden
fixtures generated from the reference and against the oracle restatement.
Integer/byte/index work: every comparison is bit-exact."""

import itertools
import random

import numpy as np
import pytest

from conftest import fromhex
from oracle import oracle as O
from sctools_amd import sharding, _lib, barcode, encodings, synthetic

pytestmark = pytest.mark.gpu

TwoBit, ThreeBit = encodings.TwoBit, encodings.ThreeBit


# ---------------------------------------------------------------- encodings vs golden
def test_encode_golden(golden):
    for rec in golden["encode"]:
        seq = bytes.fromhex(rec["seq"])
        enc = TwoBit if rec["enc"] == 2 else ThreeBit
        if "error" in rec:
            with pytest.raises(KeyError) as ei:
                enc.encode(seq)
            assert list(ei.value.args) == rec["error"]["args"]
        else:
            assert enc.encode(seq) == int(rec["code"]), rec


def test_encode_array_golden(golden):
    # batch path: group the deterministic cases by (encoder, length)
    groups = {}
    for rec in golden["encode"]:
        if "error" in rec or rec["L"] == 0:
            continue
        groups.setdefault((rec["enc"], rec["L"]), []).append(rec)
    for (kind, L), recs in groups.items():
        enc = TwoBit if kind == 2 else ThreeBit
        seqs = [bytes.fromhex(r["seq"]) for r in recs]
        codes, gc = enc.encode_array(seqs, return_gc=True)
        got = _lib.limbs_to_ints(codes.reshape(len(seqs), -1))
        assert got == [int(r["code"]) for r in recs]
        if L <= 255:
            want_gc = [s.upper().count(b"C") + s.upper().count(b"G") for s in seqs]
            assert gc.tolist() == want_gc


def test_two_bit_ambiguous_rng_order(golden):
    for case in golden["encode_ambiguous"]:
        random.seed(case["seed"])
        seqs = [bytes.fromhex(s) for s in case["seqs"]]
        got = []
        if case.get("error"):
            with pytest.raises(KeyError) as ei:
                for s in seqs:
                    got.append(str(TwoBit.encode(s)))
            assert list(ei.value.args) == case["error"]["args"]
        else:
            got = [str(TwoBit.encode(s)) for s in seqs]
        assert got == case["codes"]
        assert random.getrandbits(32) == case["after"]  # same number of draws


def test_two_bit_ambiguous_batch_matches_sequential(golden):
    for case in golden["encode_ambiguous"]:
        if case.get("error"):
            continue
        seqs = [bytes.fromhex(s) for s in case["seqs"]]
        by_len = {}
        for s in seqs:
            by_len.setdefault(len(s), []).append(s)
        for L, group in by_len.items():
            random.seed(case["seed"] + L)
            seq_codes = [TwoBit.encode(s) for s in group]
            after_seq = random.getrandbits(32)
            random.seed(case["seed"] + L)
            arr = TwoBit.encode_array(group)
            after_arr = random.getrandbits(32)
            assert _lib.limbs_to_ints(arr.reshape(len(group), -1)) == seq_codes
            assert after_seq == after_arr


def test_decode_gc_golden(golden):
    for rec in golden["decode2"]:
        t = TwoBit(rec["L"])
        code = int(rec["code"])
        assert t.decode(code) == bytes.fromhex(rec["decoded"])
        assert t.gc_content(code) == rec["gc"]
    for rec in golden["decode3"]:
        code = int(rec["code"])
        assert ThreeBit.gc_content(code) == rec["gc"]
        if "error" in rec:
            with pytest.raises(KeyError) as ei:
                ThreeBit.decode(code)
            assert list(ei.value.args) == rec["error"]["args"]
        else:
            assert ThreeBit.decode(code) == bytes.fromhex(rec["decoded"])


def test_decode_array_golden(golden):
    by_L = {}
    for rec in golden["decode2"]:
        by_L.setdefault(rec["L"], []).append(rec)
    for L, recs in by_L.items():
        codes = _lib.ints_to_limbs([int(r["code"]) for r in recs])
        t = TwoBit(L)
        assert [bytes(x) for x in t.decode_array(codes)] == [bytes.fromhex(r["decoded"]) for r in recs]
        assert t.gc_content_array(codes).tolist() == [r["gc"] for r in recs]


def test_hamming_golden(golden):
    rows = golden["hamming"]
    for a, b, d2, d3 in rows[:400]:
        assert TwoBit.hamming_distance(int(a), int(b)) == d2
        assert ThreeBit.hamming_distance(int(a), int(b)) == d3
    # batch path over all rows, grouped by limb count
    a = [int(r[0]) for r in rows]
    b = [int(r[1]) for r in rows]
    words = _lib.words_for_bits(max(max(x.bit_length() for x in a), max(x.bit_length() for x in b)))
    la, lb = _lib.ints_to_limbs(a, words), _lib.ints_to_limbs(b, words)
    assert TwoBit.hamming_distance_array(la, lb).tolist() == [r[2] for r in rows]
    assert ThreeBit.hamming_distance_array(la, lb).tolist() == [r[3] for r in rows]


def test_negative_ints_golden(golden_edges):
    """negative ints where the reference's loops end (edges.json,
    generated from the reference), scalar and batch; ValueError where they never end."""
    by_L = {}
    for rec in golden_edges["twobit_negative"]:
        t, x = TwoBit(rec["L"]), int(rec["code"])
        assert t.decode(x).hex() == rec["decode"]["bytes"], rec
        assert t.gc_content(x) == int(rec["gc"]["value"]), rec
        by_L.setdefault(rec["L"], []).append(rec)
    for L, recs in by_L.items():
        if L == 0:
            continue
        t = TwoBit(L)
        xs = [int(r["code"]) for r in recs]
        assert [bytes(v).hex() for v in t.decode_array(xs)] == [r["decode"]["bytes"] for r in recs]
        assert t.gc_content_array(xs).tolist() == [int(r["gc"]["value"]) for r in recs]
        small = [x for x in xs if x >= -(2 ** 63)]
        want = [r for r in recs if int(r["code"]) >= -(2 ** 63)]
        arr = np.array(small, dtype=np.int64)
        assert [bytes(v).hex() for v in t.decode_array(arr)] == [r["decode"]["bytes"] for r in want]
        assert t.gc_content_array(arr).tolist() == [int(r["gc"]["value"]) for r in want]
    rows = golden_edges["hamming_negative"]
    for a, b, d2, d3 in rows:
        assert TwoBit.hamming_distance(int(a), int(b)) == d2, (a, b)
        assert ThreeBit.hamming_distance(int(a), int(b)) == d3, (a, b)
    a = [int(r[0]) for r in rows]
    b = [int(r[1]) for r in rows]
    assert TwoBit.hamming_distance_array(a, b).tolist() == [r[2] for r in rows]
    assert ThreeBit.hamming_distance_array(a, b).tolist() == [r[3] for r in rows]
    i64 = [k for k, (x, y) in enumerate(zip(a, b)) if min(x, y) >= -(2 ** 63)]
    aa = np.array([a[k] for k in i64], dtype=np.int64)
    bb = np.array([b[k] for k in i64], dtype=np.int64)
    assert TwoBit.hamming_distance_array(aa, bb).tolist() == [rows[k][2] for k in i64]
    assert ThreeBit.hamming_distance_array(aa, bb).tolist() == [rows[k][3] for k in i64]
    for rec in golden_edges["threebit_decode_negative"]:
        with pytest.raises(KeyError) as ei:
            ThreeBit.decode(int(rec["code"]))
        assert list(ei.value.args) == rec["decode"]["error"]["args"], rec
    # where the reference never returns: ValueError, not a hang and not a made-up value
    for x, y in golden_edges["hangs"]["hamming_mixed_signs"]:
        for enc in (TwoBit, ThreeBit):
            with pytest.raises(ValueError):
                enc.hamming_distance(int(x), int(y))
            with pytest.raises(ValueError):
                enc.hamming_distance_array([int(x)], [int(y)])
    with pytest.raises(ValueError):
        TwoBit.hamming_distance_array(np.array([-1, 2], np.int64), np.array([-3, -4], np.int64))
    for x in golden_edges["hangs"]["threebit_gc_negative"]:
        with pytest.raises(ValueError):
            ThreeBit.gc_content(int(x))
    with pytest.raises(TypeError):
        TwoBit(4).decode(1.5)  # `1.5 & 3` is a TypeError there


def test_from_iterable_bytes_items_golden(golden_edges):
    """barcode.py:111-114 on non-bytes items: the reference's TypeError, or its codes."""
    items = {
        "ints": [5, 6], "int_after_bytes": [b"ACGT", 7], "str": ["ACGT"], "empty_str": [""],
        "list_of_ints": [[65, 67, 71, 84], [84, 84, 65, 65]],
        "bytearray": [bytearray(b"ACGT"), memoryview(b"TTGA")], "tuple_of_ints": [(65, 67)],
        "none": [None], "float": [1.5]}
    for rec in golden_edges["from_iterable_bytes"]:
        its = items[rec["name"]]
        if "error" in rec:
            with pytest.raises(TypeError) as ei:
                barcode.Barcodes.from_iterable_bytes(its, rec["L"])
            assert list(ei.value.args) == rec["error"]["args"], rec
        else:
            s = barcode.Barcodes.from_iterable_bytes(its, rec["L"])
            assert [str(k) for k in s] == rec["codes"] and [s[k] for k in s] == rec["counts"]


def test_from_iterable_strings_items_golden(golden_edges):
    """barcode.py:104-108 item by item: the first failing item's error (or an earlier item's
    KeyError) after exactly the draws the reference makes, or its codes; the RNG state after
    the call matches the reference's."""
    import builtins
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from gen_golden_edges import iterable_from_spec
    for rec in golden_edges["from_iterable_strings"]:
        random.seed(rec["seed"])
        its = iterable_from_spec(rec["spec"])
        if "error" in rec:
            with pytest.raises(getattr(builtins, rec["error"]["type"])) as ei:
                barcode.Barcodes.from_iterable_strings(its, rec["L"])
            assert type(ei.value).__name__ == rec["error"]["type"], rec["name"]
            assert list(ei.value.args) == rec["error"]["args"], rec["name"]
        else:
            s = barcode.Barcodes.from_iterable_strings(its, rec["L"])
            assert [str(k) for k in s] == rec["codes"] and [s[k] for k in s] == rec["counts"], rec["name"]
        assert random.getrandbits(32) == rec["after"], rec["name"]


def test_reference_simple_barcodes(golden):
    sb = golden["simple_barcodes"]
    seqs = [bytes.fromhex(s) for s in sb["seqs"]]
    import itertools
    for enc, key in ((TwoBit, "two"), (ThreeBit, "three")):
        e = enc(4)
        codes = [e.encode(s) for s in seqs]
        assert [e.hamming_distance(x, y) for x, y in itertools.combinations(codes, 2)] == sb[key]


def test_reference_roundtrips():
    # test_encodings.py:27-59 on the drop-in
    seq = b'ACGTTTGAGATGAGATATAGANNNN'
    t2 = TwoBit(len(seq))
    assert t2.decode(t2.encode(seq))[:4] == seq[:4]
    assert ThreeBit.decode(ThreeBit.encode(seq)) == seq
    s = b'AGCGCGAT'
    assert t2.gc_content(t2.encode(s)) == s.count(b'C') + s.count(b'G')
    assert ThreeBit.gc_content(ThreeBit.encode(seq)) == seq.count(b'C') + seq.count(b'G')
    with pytest.raises(KeyError):
        t2.encode(b'ACGTP')
    assert ThreeBit.decode(ThreeBit.encode(b'ACGTP')) == b'ACGTN'


# ---------------------------------------------------------------- barcode sets vs golden
def test_whitelist_1k(golden, tmp_path):
    wl = golden["whitelist_1k"]
    codes = [int(c) for c in wl["codes"]]
    p = tmp_path / "1k.txt"
    p.write_bytes(b"".join(TwoBit(16).decode(c) + b"\n" for c in codes))
    bset = barcode.Barcodes.from_whitelist(str(p), 16)
    assert list(bset) == codes
    assert bset.hamming_histogram().astype(np.int64).tolist() == wl["hist"]
    summ = bset.summarize_hamming_distances()
    assert summ == fromhex(wl["summary"])
    assert all(isinstance(v, np.float64) for v in summ.values())
    assert bset.base_frequency().tolist() == wl["base_frequency"]
    assert [float(x) for x in bset.effective_diversity()] == [float.fromhex(x) for x in wl["effective_diversity"]]


def test_first50_and_encoded(golden):
    for mode, rec in golden["first50"].items():
        codes = [int(c) for c in rec["codes"]]
        s = barcode.ObservedBarcodeSet.from_iterable_encoded(codes, 16)
        assert s.summarize_hamming_distances() == fromhex(rec["summary"])
        seqs = [TwoBit(16).decode(c) for c in codes]
        if mode == "bytes":
            s2 = barcode.Barcodes.from_iterable_bytes(seqs, 16)
        else:
            s2 = barcode.Barcodes.from_iterable_strings([x.decode() for x in seqs], 16)
        assert list(s2) == codes
    rec = golden["encoded_0_7"]
    s = barcode.Barcodes.from_iterable_encoded([0, 1, 2, 3, 4, 5, 6, 7], barcode_length=2)
    assert [TwoBit(2).decode(b).hex() for b in s] == rec["decoded"]
    assert s.summarize_hamming_distances() == fromhex(rec["summary"])


def test_small_sets_summary(golden):
    for rec in golden["small_sets"]:
        s = barcode.Barcodes.from_iterable_encoded([int(c) for c in rec["codes"]], rec["L"])
        if rec["error"]:
            with pytest.raises(IndexError) as ei:
                s.summarize_hamming_distances()
            assert list(ei.value.args) == rec["error"]["args"]
        else:
            assert s.summarize_hamming_distances() == fromhex(rec["summary"]), rec


def test_errors(golden):
    with pytest.raises(IndexError):
        barcode.Barcodes.from_iterable_encoded([5], barcode_length=4).summarize_hamming_distances()
    with pytest.raises(TypeError) as ei:
        barcode.Barcodes([1, 2, 3], 4)
    assert list(ei.value.args) == golden["errors"]["not_mapping"]["args"]


def test_config1_10k(golden_10k):
    n, L, seed = golden_10k["n"], golden_10k["L"], golden_10k["seed"]
    codes = synthetic.whitelist_codes(n, L, seed)
    s = barcode.PriorBarcodeSet.from_iterable_encoded(codes.tolist(), L)
    assert s.hamming_histogram().astype(np.int64).tolist() == golden_10k["hist"]
    assert s.summarize_hamming_distances() == fromhex(golden_10k["summary"])


# ---------------------------------------------------------------- all-pairs kernel vs oracle
@pytest.mark.parametrize("n", [2, 3, 31, 32, 33, 63, 64, 65, 255, 256, 257, 511, 512, 513,
                               1023, 1024, 1025, 2047, 2049, 4100])
def test_allpairs_sizes(n):
    rng = np.random.default_rng(n)
    codes = np.unique(rng.integers(0, 2 ** 32, size=n + 64, dtype=np.uint64))[:n]
    rng.shuffle(codes)
    hist = _lib.hamming_hist_allpairs(codes, 32)
    ref = O.c_hist_rows(codes)[: hist.size]
    assert hist.astype(np.int64).tolist() == ref.tolist()
    assert int(hist.sum()) == n * (n - 1) // 2


@pytest.mark.parametrize("bits", list(range(1, 65)))
def test_allpairs_code_widths(bits):
    rng = np.random.default_rng(bits)
    hi = 2 ** bits
    n = min(hi, 1500)
    codes = np.unique(rng.integers(0, hi, size=n, dtype=np.uint64, endpoint=False)) if bits < 64 else \
        np.unique(rng.integers(0, 2 ** 63, size=n, dtype=np.uint64) * np.uint64(2) + np.uint64(1))
    hist = _lib.hamming_hist_allpairs(codes)
    ref = O.c_hist_rows(codes)
    nb = hist.size
    assert hist.astype(np.int64).tolist() == ref[:nb].tolist()
    assert ref[nb:].sum() == 0


def test_allpairs_duplicates_and_clusters():
    # duplicates give distance 0; clustered codes exercise every low bin
    base = synthetic.whitelist_codes(700, 16, seed=3)
    near = base ^ (np.uint64(1) << (np.arange(700, dtype=np.uint64) % np.uint64(32)))
    codes = np.concatenate([base, near, base[:50]])
    hist = _lib.hamming_hist_allpairs(codes, 32)
    ref = O.c_hist_rows(codes)[:17]
    assert hist.astype(np.int64).tolist() == ref.tolist()
    assert hist[0] >= 50


def test_allpairs_shards_sum_to_whole():
    torch = pytest.importorskip("torch")
    codes = synthetic.whitelist_codes(20_000, 16, seed=9)
    d_codes = torch.from_numpy(codes.view(np.int64)).cuda()
    # per-range inversion needs self-contained counts: the SUBSETS scheme
    plan = _lib.AllPairsPlan(d_codes.data_ptr(), codes.size, 32, scheme=_lib.SCHEME_SUBSETS)
    assert plan.scheme == _lib.SCHEME_SUBSETS and plan.ncounts == plan.nbins
    plan.build()
    full = torch.zeros(plan.nbins, dtype=torch.int64, device="cuda")
    plan.count(full.data_ptr())
    parts = torch.zeros(plan.nbins, dtype=torch.int64, device="cuda")
    cuts = [0, 7, plan.items // 3, plan.items // 2 + 5, plan.items - 1, plan.items]
    total_pairs = 0
    for b, e in zip(cuts[:-1], cuts[1:]):
        one = torch.zeros(plan.nbins, dtype=torch.int64, device="cuda")
        plan.count(one.data_ptr(), b, e, grid=37)
        torch.cuda.synchronize()
        pairs = plan.range_pairs(b, e)
        ref = np.zeros(65, dtype=np.int64)
        np_ = np.zeros(1, dtype=np.int64)
        O.c_oracle().oracle_hist_items(codes.ctypes.data, codes.size, 256, 1024, ref.ctypes.data,
                                       b, e, np_.ctypes.data, 0)
        assert int(one[0].item()) == pairs == int(np_[0])
        hist_one = _lib.counts_to_hist(one.cpu().numpy().view(np.uint64))
        assert hist_one.astype(np.int64).tolist() == ref[: plan.nbins].tolist()
        parts += one
        total_pairs += pairs
    torch.cuda.synchronize()
    assert torch.equal(full, parts)
    assert total_pairs == plan.pairs == codes.size * (codes.size - 1) // 2
    plan.close()


@pytest.mark.parametrize("scheme", [0, 1])
def test_allpairs_partial_builds_per_rank(scheme):
    """Each 'rank' builds only the table chunks of its item range (build_items), counts that
    range and its moment share; the summed counts invert to the oracle histogram."""
    torch = pytest.importorskip("torch")
    codes = synthetic.whitelist_codes(30_000, 16, seed=21)
    d_codes = torch.from_numpy(codes.view(np.int64)).cuda()
    world = 3
    total = None
    for rank in range(world):
        plan = _lib.AllPairsPlan(d_codes.data_ptr(), codes.size, 32, scheme=scheme)
        b, e = sharding.item_range(plan.items, rank, world)
        c = torch.zeros(plan.ncounts, dtype=torch.int64, device="cuda")
        plan.build(0, b, e)
        plan.moments(c.data_ptr(), rank, world)
        plan.count(c.data_ptr(), b, e)
        total = c if total is None else total + c
        sch, nb = plan.scheme, plan.nbins
        plan.close()
    hist = _lib.counts_to_hist(total.cpu().numpy().view(np.uint64), sch, nb)
    assert hist.astype(np.int64).tolist() == O.c_hist_rows(codes)[:17].tolist()


def test_allpairs_737k_properties():
    """Full config-2 size: size-independent checks, the three count schemes agree, and
    exact parity on a 60k-code prefix."""
    torch = pytest.importorskip("torch")
    n, L, seed = synthetic.CONFIGS[2]
    codes = synthetic.whitelist_codes(n, L, seed)
    d_codes = torch.from_numpy(codes.view(np.int64)).cuda()
    hists = {}
    for scheme in (_lib.SCHEME_MOMENTS, _lib.SCHEME_SUBSETS, _lib.SCHEME_SPECTRAL):
        plan = _lib.AllPairsPlan(d_codes.data_ptr(), n, 32, scheme=scheme)
        assert plan.scheme == scheme
        plan.build()
        counts = torch.zeros(plan.ncounts, dtype=torch.int64, device="cuda")
        plan.moments(counts.data_ptr())
        plan.count(counts.data_ptr())
        c = counts.cpu().numpy().view(np.uint64)
        assert int(c[0]) == (n if scheme == _lib.SCHEME_SPECTRAL else n * (n - 1) // 2)
        hist = plan.counts_to_hist(c)
        assert int(hist.sum()) == n * (n - 1) // 2
        # twice gives the same (integer atomics are order independent)
        counts2 = torch.zeros_like(counts)
        plan.moments(counts2.data_ptr())
        plan.count(counts2.data_ptr(), grid=333)
        assert torch.equal(counts, counts2)
        hists[scheme] = hist.tolist()
        plan.close()
    assert hists[_lib.SCHEME_MOMENTS] == hists[_lib.SCHEME_SUBSETS] == hists[_lib.SCHEME_SPECTRAL]
    # the mean distance is fixed by the per-position base counts alone (first moment)
    bases = (codes[:, None] >> (2 * np.arange(16, dtype=np.uint64))) & np.uint64(3)
    agree = sum(int(np.bincount(bases[:, p].astype(np.int64), minlength=4).astype(object).dot(
        np.bincount(bases[:, p].astype(np.int64), minlength=4).astype(object) - 1)) // 2 for p in range(16))
    h = hists[_lib.SCHEME_MOMENTS]
    assert sum(d * x for d, x in enumerate(h)) == 16 * (n * (n - 1) // 2) - agree
    # exact parity on a 60k prefix
    sub = codes[:60_000]
    hs = _lib.hamming_hist_allpairs(sub, 32)
    ref = O.c_hist_rows(sub)[:17]
    assert hs.astype(np.int64).tolist() == ref.tolist()


@pytest.mark.parametrize("n", [2, 3, 5, 64, 255, 1025, 4100, 20_000])
def test_allpairs_moments_scheme_matches_oracle(n):
    """MOMENTS scheme (13 products + agreement moments) vs the C oracle, including
    duplicates (d = 0) and complementary codes (d = 16), which share d mod 16 = 0."""
    torch = pytest.importorskip("torch")
    codes = synthetic.whitelist_codes(max(2, n - n // 8), 16, seed=n)
    extra = []
    if n >= 5:
        extra = [codes[0], codes[1] ^ np.uint64(0xAAAAAAAA), codes[1] ^ np.uint64(0xFFFFFFFF)]
    codes = np.concatenate([codes, np.array(extra, dtype=np.uint64)])[:max(n, 2)]
    d_codes = torch.from_numpy(codes.view(np.int64)).cuda()
    plan = _lib.AllPairsPlan(d_codes.data_ptr(), codes.size, 32, scheme=_lib.SCHEME_MOMENTS)
    plan.build()
    counts = torch.zeros(plan.ncounts, dtype=torch.int64, device="cuda")
    for part in range(3):  # moment shares, as three ranks would add them
        plan.moments(counts.data_ptr(), part, 3)
    items = plan.items
    for b, e in ((0, items // 2), (items // 2, items)):
        plan.count(counts.data_ptr(), b, e, grid=29)
    hist = plan.counts_to_hist(counts.cpu().numpy().view(np.uint64))
    ref = O.c_hist_rows(codes)[:17]
    assert hist.astype(np.int64).tolist() == ref.tolist()
    # the one-shot host entry point picks MOMENTS for 16-base codes
    assert _lib.hamming_hist_allpairs(codes, 32).astype(np.int64).tolist() == ref.tolist()
    plan.close()


def _spectral_hist(codes, ranges=None, chunk=None):
    torch = pytest.importorskip("torch")
    d_codes = torch.from_numpy(codes.view(np.int64)).cuda()
    with _lib.tuning(spectral_chunk=chunk):
        plan = _lib.AllPairsPlan(d_codes.data_ptr(), codes.size, 32, scheme=_lib.SCHEME_SPECTRAL)
    try:
        assert plan.scheme == _lib.SCHEME_SPECTRAL and plan.ncounts == 53
        assert plan.items == (1 << 18 if codes.size >= 2 else 0)
        counts = torch.zeros(plan.ncounts, dtype=torch.int64, device="cuda")
        items = plan.items
        if ranges is None:
            ranges = [(0, items)]
        credited = 0
        for b, e in ranges:  # as separate ranks would: each builds, then counts its slices
            plan.build(0, b, e)
            plan.count(counts.data_ptr(), b, e)
            credited += plan.range_pairs(b, e)
        assert credited == codes.size * (codes.size - 1) // 2
        c = counts.cpu().numpy().view(np.uint64)
        assert int(c[0]) == (codes.size if codes.size >= 2 else 0)
        return plan.counts_to_hist(c)
    finally:
        plan.close()


@pytest.mark.parametrize("n", [2, 3, 5, 1025, 20_000])
def test_allpairs_spectral_scheme_matches_oracle(n):
    """SPECTRAL scheme (Walsh-Hadamard transform over Z_2^32, no pair enumerated) vs the
    C oracle, with duplicates (d = 0) and complementary codes (d = 16), counted in three
    slice ranges."""
    codes = synthetic.whitelist_codes(max(2, n - n // 8), 16, seed=n + 7)
    extra = []
    if n >= 5:
        extra = [codes[0], codes[0], codes[1] ^ np.uint64(0xAAAAAAAA), codes[1] ^ np.uint64(0xFFFFFFFF)]
    codes = np.concatenate([codes, np.array(extra, dtype=np.uint64)])[:max(n, 2)]
    hist = _spectral_hist(codes, [(0, 1000), (1000, 1001), (1001, 1 << 18)])
    assert hist.astype(np.int64).tolist() == O.c_hist_rows(codes)[:17].tolist()


@pytest.mark.parametrize("dense", [200, 33_000])
def test_allpairs_spectral_wide_intermediates(dense):
    """A transform column (low 14 bits) of `dense` codes makes the seed -> tile intermediate
    int16 (> 127 codes) or int32 (> 32,767): the VALU tile kernel on both, next to 3,000
    sparse codes, duplicates and complements, in two slice ranges with 1000-slice chunks."""
    rng = np.random.default_rng(dense)
    hi = rng.choice(1 << 18, dense, replace=False).astype(np.uint64)
    col = (hi << np.uint64(14)) | np.uint64(0x2345)
    rest = synthetic.whitelist_codes(3000, 16, seed=dense + 1)
    rest = rest[(rest & np.uint64(0x3FFF)) != np.uint64(0x2345)]
    codes = np.concatenate([col, rest, col[:3], rest[:2] ^ np.uint64(0xFFFFFFFF)])
    rng.shuffle(codes)
    hist = _spectral_hist(codes, [(0, 4099), (4099, 1 << 18)], chunk=1000 if dense < 1000 else None)
    assert hist.astype(np.int64).tolist() == O.c_hist16(codes)[0][:17].tolist()


def test_allpairs_spectral_chunk_seams():
    """The shipped seed / tile kernels with 1000-slice chunks (seams inside Gray walks and
    inside the tile's digit-weight runs) and a range cut at 777."""
    codes = synthetic.whitelist_codes(30_000, 16, seed=5)
    codes = np.concatenate([codes, codes[:3], codes[3:5] ^ np.uint64(0xFFFFFFFF)])
    hist = _spectral_hist(codes, [(0, 777), (777, 1 << 18)], chunk=1000)
    assert hist.astype(np.int64).tolist() == O.c_hist_rows(codes)[:17].tolist()


def test_allpairs_spectral_column_sizes():
    """Columns (low 14 bits) holding 63, 64, 65, 100 and 127 codes -- two and four 32-code
    plane groups (one and two register-resident, the rest from L2) and the int8 limit --
    next to sparse ones, duplicates included; slice ranges cut inside walks."""
    rng = np.random.default_rng(21)
    bg = synthetic.whitelist_codes(5000, 16, seed=3)
    cols = (5, 6, 7, 20, 16383)
    parts = [bg[~np.isin(bg & np.uint64(0x3FFF), np.array(cols, dtype=np.uint64))]]
    for col, m in zip(cols, (63, 64, 65, 100, 127)):
        hi = rng.integers(0, 1 << 18, m).astype(np.uint64)
        hi[-1] = hi[0]  # a duplicate code inside the column
        parts.append((hi << np.uint64(14)) | np.uint64(col))
    codes = np.concatenate(parts)
    hist = _spectral_hist(codes, [(0, 300), (300, 8191), (8191, 1 << 18)])
    assert hist.astype(np.int64).tolist() == O.c_hist_rows(codes)[:17].tolist()


def test_allpairs_spectral_high_energy_planes():
    """Planes (column bits 12, 13) of large seeds in every slice -- 120 columns of 120 codes,
    110 of them sharing their high bits, in planes 0 and 2 -- beside sparse ones (squares
    above 2^32 per plane, |G| above 2^16, the packed int16 plane sums near their range)."""
    rng = np.random.default_rng(33)
    bg = synthetic.whitelist_codes(5000, 16, seed=8)
    parts = []
    dense = np.concatenate([rng.choice(4096, 120, replace=False), 8192 + rng.choice(4096, 120, replace=False)])
    bg = bg[~np.isin(bg & np.uint64(0x3FFF), dense.astype(np.uint64))]
    parts.append(bg)
    for col in dense:
        hi = np.full(120, rng.integers(0, 1 << 18), dtype=np.uint64)
        hi[110:] = rng.integers(0, 1 << 18, 10).astype(np.uint64)
        parts.append((hi << np.uint64(14)) | np.uint64(col))
    codes = np.concatenate(parts)
    hist = _spectral_hist(codes, [(0, 5000), (5000, 1 << 18)])
    assert hist.astype(np.int64).tolist() == O.c_hist_rows(codes)[:17].tolist()


def test_allpairs_spectral_crowded_low_bits():
    """3000 codes sharing their low 14 bits (one transform column holds them all: 94
    32-code groups of bit planes, an int16 intermediate), plus codes that differ only
    there, with a 300-slice chunk (Gray walks cut by chunk seams)."""
    rng = np.random.default_rng(11)
    hi = rng.integers(0, 1 << 12, 3000).astype(np.uint64)
    codes = (hi << np.uint64(20)) | np.uint64(0x5A5A5)
    codes = np.concatenate([codes, codes[:20] ^ np.uint64(0xFFFFF), rng.integers(0, 1 << 32, 50).astype(np.uint64)])
    hist = _spectral_hist(codes, [(0, 1 << 18)], chunk=300)
    assert hist.astype(np.int64).tolist() == O.c_hist_rows(codes)[:17].tolist()


def test_allpairs_spectral_is_auto_for_large_whitelists():
    """The one-shot host entry point resolves AUTO to SPECTRAL at config-5 scale and agrees
    with the MOMENTS count kernel on a 1.6M-code whitelist."""
    torch = pytest.importorskip("torch")
    codes = synthetic.whitelist_codes(1_600_000, 16, 99)
    d_codes = torch.from_numpy(codes.view(np.int64)).cuda()
    auto = _lib.AllPairsPlan(d_codes.data_ptr(), codes.size, 32)
    assert auto.scheme == _lib.SCHEME_SPECTRAL
    auto.close()
    hs = _lib.hamming_hist_allpairs(codes, 32)
    mom = _lib.AllPairsPlan(d_codes.data_ptr(), codes.size, 32, scheme=_lib.SCHEME_MOMENTS)
    mom.build()
    counts = torch.zeros(mom.ncounts, dtype=torch.int64, device="cuda")
    mom.moments(counts.data_ptr())
    mom.count(counts.data_ptr())
    hm = mom.counts_to_hist(counts.cpu().numpy().view(np.uint64))
    mom.close()
    assert hs.tolist() == hm.tolist()


def test_plan_cache_reuse_and_release():
    """The plan cache (sct_allpairs_cache_release, SCT_TUNE_PLAN_CACHE): one-shot calls on sets
    of different sizes and seed widths reuse (and grow) the device's cached buffers; a plan
    created while another holds the cache owns its buffers; a plan counted on a side stream and
    destroyed hands the cache to the next plan only after its work is done; release and the
    cache switched off give the same histograms.  Each against the C oracle."""
    torch = pytest.importorskip("torch")
    sets = [synthetic.whitelist_codes(n, 16, seed=n) for n in (400_000, 2_000, 350_000)]
    sets.append(np.concatenate([sets[1], np.repeat(sets[1][:3], 200)]))  # forced SPECTRAL: int16 seeds
    refs = [O.c_hist16(c)[0][:17].tolist() for c in sets]
    for c, ref in zip(sets, refs):  # AUTO: SPECTRAL, MOMENTS, SPECTRAL, MOMENTS
        assert _lib.hamming_hist_allpairs(c, 32).astype(np.int64).tolist() == ref
    for c, ref in zip(sets, refs):  # forced SPECTRAL at every size
        assert _spectral_hist(c).astype(np.int64).tolist() == ref
    # a live plan holds the cache: a second plan meanwhile owns its buffers
    d0 = torch.from_numpy(sets[0].view(np.int64)).cuda()
    holder = _lib.AllPairsPlan(d0.data_ptr(), sets[0].size, 32, scheme=_lib.SCHEME_SPECTRAL)
    assert _spectral_hist(sets[2]).astype(np.int64).tolist() == refs[2]
    # the holder counts on a side stream and is destroyed without a host sync
    side = torch.cuda.Stream()
    counts = torch.zeros(holder.ncounts, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    holder.build(side.cuda_stream)
    holder.count(counts.data_ptr(), stream=side.cuda_stream)
    holder.close()
    side.synchronize()
    assert holder.counts_to_hist(counts.cpu().numpy().view(np.uint64)).astype(np.int64).tolist() == refs[0]
    assert _spectral_hist(sets[2]).astype(np.int64).tolist() == refs[2]
    _lib.release_plan_cache()
    assert _lib.hamming_hist_allpairs(sets[0], 32).astype(np.int64).tolist() == refs[0]
    with _lib.tuning(plan_cache=0):
        assert _lib.hamming_hist_allpairs(sets[2], 32).astype(np.int64).tolist() == refs[2]
    _lib.release_plan_cache()


def test_distinct_promise_skips_sort_and_is_checked():
    """SCT_ALLPAIRS_DISTINCT (Barcodes' mapping keys): SPECTRAL takes sum f^2 = n without its
    sort; the histogram still matches the oracle, and a set that breaks the promise (one
    duplicate among 400K codes) raises ValueError from the host's exact check instead of
    returning a histogram -- with and without the promise the honest path stays exact."""
    codes = synthetic.whitelist_codes(400_000, 16, seed=77)
    ref = O.c_hist16(codes)[0][:17].tolist()
    assert _lib.hamming_hist_allpairs(codes, 32, distinct=True).astype(np.int64).tolist() == ref
    dup = codes.copy()
    dup[-1] = dup[0]
    with pytest.raises(ValueError, match="sum f"):
        _lib.hamming_hist_allpairs(dup, 32, distinct=True)
    assert _lib.hamming_hist_allpairs(dup, 32).astype(np.int64).tolist() == O.c_hist16(dup)[0][:17].tolist()
    b = barcode.Barcodes({int(c): 1 for c in codes}, 16)
    assert b.hamming_histogram().astype(np.int64).tolist() == ref


def _heavy_multiset(case):
    """Observed-barcode multisets whose sum f^2 exceeds 2^32 (so sum_w S_w = 2^32 sum f^2
    exceeds 2^64): shuffled, with the seed width they force."""
    rng = np.random.default_rng({"one_heavy": 1, "zipf": 2, "int16_heavy": 3}[case])
    if case == "one_heavy":  # 330K unique codes + one of them 70K times more (int32 seeds)
        wl = synthetic.whitelist_codes(330_000, 16, seed=41)
        codes, width = np.concatenate([wl, np.full(70_000, wl[12345], dtype=np.uint64)]), 4
    elif case == "zipf":  # 400K cells, multiplicity ~ 80000 / rank^1.3 (int32 seeds)
        wl = synthetic.whitelist_codes(400_000, 16, seed=42)
        rng.shuffle(wl)
        f = np.maximum(1, (80_000 / np.arange(1, wl.size + 1) ** 1.3).astype(np.int64))
        codes, width = np.repeat(wl, f), 4
    else:  # 8 codes x 30,000 in 8 columns (<= 32,767 codes each: int16 seeds) + 400K unique
        wl = synthetic.whitelist_codes(400_008, 16, seed=43)
        codes, width = np.concatenate([wl, np.repeat(wl[:8], 29_999)]), 2
    rng.shuffle(codes)
    _, f = np.unique(codes, return_counts=True)
    assert int((f.astype(np.int64) ** 2).sum()) >= 1 << 32
    return codes, width


@pytest.mark.parametrize("case", ["one_heavy", "zipf", "int16_heavy"])
def test_allpairs_spectral_heavy_multisets_bin_for_bin(case):
    """SPECTRAL on multisets with sum f^2 >= 2^32: the weight sums exceed
    2^64 in total, so the device accumulates them in non-carrying limbs and the host checks
    sum_w S_w == 2^32 sum f^2 against the sorted-code count.  Forced SPECTRAL over two slice
    ranges, AUTO through the one-shot host entry point, and the product's sharded driver, each
    bin for bin against the C oracle's pair loop (encodings.py:113-121: equal codes are
    distance 0)."""
    torch = pytest.importorskip("torch")
    codes, width = _heavy_multiset(case)
    ref, _ = O.c_hist16(codes)
    ref = ref[:17].tolist()
    d_codes = torch.from_numpy(codes.view(np.int64)).cuda()
    plan = _lib.AllPairsPlan(d_codes.data_ptr(), codes.size, 32, scheme=_lib.SCHEME_SPECTRAL)
    try:
        assert plan.spectral_info()["elem_bytes"] == width
    finally:
        plan.close()
    assert _spectral_hist(codes, [(0, 70_001), (70_001, 1 << 18)]).astype(np.int64).tolist() == ref
    assert codes.size >= 325_000  # AUTO = SPECTRAL
    assert _lib.hamming_hist_allpairs(codes, 32).astype(np.int64).tolist() == ref
    assert sharding.allpairs_histogram_sharded(codes, 32).astype(np.int64).tolist() == ref


# ---------------------------------------------------------------- nearest whitelist
def test_nearest_golden(golden):
    for name, enc in (("three", "ThreeBit"), ("two", "TwoBit")):
        rec = golden["nearest"][name]
        wl = np.array([int(c) for c in rec["whitelist"]], dtype=np.uint64)
        q = np.array([int(c) for c in rec["queries"]], dtype=np.uint64)
        for md, want in rec["result"].items():
            idx, dist = barcode.nearest_whitelist(q, wl, max_distance=int(md), encoding=enc)
            assert idx.tolist() == want["index"], (name, md)
            assert dist.tolist() == want["dist"], (name, md)


def _config4_queries(wl_seqs, nq, rng, alphabet=b"ACGT"):
    """50% exact whitelist draws, 25% one substitution, 15% one N, 10% random."""
    L = wl_seqs.shape[1]
    picks = wl_seqs[rng.integers(0, wl_seqs.shape[0], nq)].copy()
    kind = rng.random(nq)
    pos = rng.integers(0, L, nq)
    sub = (kind >= 0.5) & (kind < 0.75)
    picks[sub, pos[sub]] = np.frombuffer(alphabet, np.uint8)[rng.integers(0, len(alphabet), sub.sum())]
    nn = (kind >= 0.75) & (kind < 0.9)
    picks[nn, pos[nn]] = ord("N")
    rnd = kind >= 0.9
    picks[rnd] = np.frombuffer(alphabet, np.uint8)[rng.integers(0, len(alphabet), (rnd.sum(), L))]
    return picks


_NEAREST_SCHEMES = {"auto": _lib.NEAREST_AUTO, "oa": _lib.NEAREST_OA, "csr": _lib.NEAREST_CSR,
                    "halves": _lib.NEAREST_HALVES}


@pytest.mark.parametrize("scheme", ["auto", "csr", "oa", "halves"])
@pytest.mark.parametrize("kind,max_d", [(3, 0), (3, 1), (3, 2), (3, 3), (2, 0), (2, 1), (2, 2)])
def test_nearest_vs_bruteforce(kind, max_d, scheme):
    """Every index scheme (CSR buckets per block; open-addressing tables of block-pair
    keys) against the brute force on config-4-shaped sets."""
    with _lib.tuning(nearest_scheme=_NEAREST_SCHEMES[scheme]):
        _nearest_vs_bruteforce(kind, max_d)


@pytest.mark.parametrize("kind,L", [(3, 16), (2, 16), (3, 15), (2, 13), (3, 7), (2, 2)])
@pytest.mark.parametrize("max_d", [0, 1])
def test_nearest_halves_edges(kind, L, max_d):
    """The half-key tables (max_d <= 1, A/C/G/T whitelists) against the brute force: odd and
    short lengths, duplicated whitelist codes (ties at 0 and at 1), queries with N or invalid
    triplets (0, 5, 7) in one or both halves, queries with bits above the whitelist's width
    (every distance shifted by the same excess), and queries 1 away from two codes."""
    rng = np.random.default_rng(1000 * kind + 10 * L + max_d)
    n = min(4 ** L, 5000)
    wl2 = synthetic.whitelist_codes(n, L, seed=L + kind)
    wl = wl2 if kind == 2 else synthetic.two_to_three(wl2, L)
    wl = np.concatenate([wl, wl[:7]])  # duplicates
    picks = wl[rng.integers(0, wl.size, 3000)]
    q = picks.copy()
    pos = rng.integers(0, L, q.size).astype(np.uint64)
    w = np.uint64(kind)
    sub = rng.integers(0, 4, q.size).astype(np.uint64) + (np.uint64(1) if kind == 3 else np.uint64(0))
    m = rng.random(q.size)
    one = m < 0.3  # one substituted base (may equal the original)
    q[one] = (q[one] & ~(np.uint64((1 << kind) - 1) << (w * pos[one]))) | (sub[one] << (w * pos[one]))
    if kind == 3:
        bad = (m >= 0.3) & (m < 0.5)  # one N / 0 / 5 / 7 triplet
        val = rng.choice(np.array([0, 5, 6, 7], dtype=np.uint64), q.size)
        q[bad] = (q[bad] & ~(np.uint64(7) << (w * pos[bad]))) | (val[bad] << (w * pos[bad]))
        two = (m >= 0.5) & (m < 0.6)  # invalid triplets in both halves
        q[two] = (q[two] & ~(np.uint64(7) << np.uint64(0))) | np.uint64(6)
        q[two] = (q[two] & ~(np.uint64(7) << (w * np.uint64(L - 1)))) | (np.uint64(6) << (w * np.uint64(L - 1)))
    hi = (m >= 0.6) & (m < 0.7)  # a non-zero group above the whitelist's width
    top = min(63, kind * L + int(rng.integers(0, 3)))
    q[hi] |= np.uint64(1) << np.uint64(top)
    rnd = m >= 0.95
    q[rnd] = rng.integers(0, 1 << min(63, kind * L), rnd.sum(), dtype=np.uint64)
    with _lib.tuning(nearest_scheme=_lib.NEAREST_HALVES):
        idx, dist = barcode.nearest_whitelist(q, wl, max_distance=max_d, encoding=kind)
    ridx, rdist = O.c_nearest(kind, wl, q, max_d)
    assert np.array_equal(idx, ridx) and np.array_equal(dist, rdist)
    if L >= 2:  # the plan really took the half-key layout
        import torch
        d_wl = torch.from_numpy(wl.view(np.int64)).cuda()
        with _lib.tuning(nearest_scheme=_lib.NEAREST_HALVES):
            plan = _lib.NearestPlan(kind, d_wl.data_ptr(), wl.size, kind * L, max_d)
        assert plan.info()["scheme"] == "halves"
        # outputs at an offset that is not 16-B aligned (the index pass's scalar path)
        d_q = torch.from_numpy(q.view(np.int64)).cuda()
        out_i = torch.full((q.size + 3,), 7, dtype=torch.int32, device="cuda")
        out_d = torch.zeros(q.size + 3, dtype=torch.uint8, device="cuda")
        plan.query(d_q.data_ptr(), q.size, out_i[1:].data_ptr(), out_d[1:].data_ptr())
        torch.cuda.synchronize()
        assert out_i[1:q.size + 1].cpu().numpy().tolist() == ridx.tolist() and int(out_i[0]) == 7
        assert out_d[1:q.size + 1].cpu().numpy().tolist() == rdist.tolist()
        plan.close()


@pytest.mark.parametrize("kind", [2, 3])
def test_nearest_halves_big_buckets(kind):
    """Buckets of many chunks (every whitelist code sharing its high half, or its low half, with
    hundreds of others: full chunks, a partial last chunk, empty buckets between) and buckets of
    exactly 16 / 17 / 32 / 33 codes, against the brute force."""
    rng = np.random.default_rng(77 + kind)
    L = 16
    hi = np.uint64(0x5A5A) << np.uint64(16)  # one high half (A key) for 700 codes
    lo_codes = np.unique(rng.integers(0, 1 << 16, 1200, dtype=np.uint64))[:700]
    wl2 = [hi | lo_codes]
    for k, size in enumerate((16, 17, 32, 33, 1)):  # buckets of exact group multiples and one more
        a = np.uint64(0x1000 + k) << np.uint64(16)
        wl2.append(a | np.unique(rng.integers(0, 1 << 16, 4 * size, dtype=np.uint64))[:size])
    b = np.uint64(0x0F0F)  # one low half (B key) for 300 codes
    wl2.append((np.unique(rng.integers(0, 1 << 16, 600, dtype=np.uint64))[:300] << np.uint64(16)) | b)
    wl2 = np.unique(np.concatenate(wl2))
    wl = wl2 if kind == 2 else synthetic.two_to_three(wl2, L)
    picks = wl[rng.integers(0, wl.size, 4000)]
    pos = rng.integers(0, L, picks.size).astype(np.uint64)
    w = np.uint64(kind)
    sub = rng.integers(0, 4, picks.size).astype(np.uint64) + (np.uint64(1) if kind == 3 else np.uint64(0))
    one = rng.random(picks.size) < 0.5
    q = picks.copy()
    q[one] = (q[one] & ~(np.uint64((1 << kind) - 1) << (w * pos[one]))) | (sub[one] << (w * pos[one]))
    ridx, rdist = O.c_nearest(kind, wl, q, 1)
    with _lib.tuning(nearest_scheme=_lib.NEAREST_HALVES):
        idx, dist = barcode.nearest_whitelist(q, wl, max_distance=1, encoding=kind)
    assert np.array_equal(idx, ridx) and np.array_equal(dist, rdist)


@pytest.mark.parametrize("kind", [3, 2])
def test_nearest_halves_sorted_and_shuffled_whitelists(kind):
    """A whitelist in alphabetical order (key order: the query kernel writes whitelist indices and
    reads the permutation only for B-table winners, no index pass) and the same whitelist shuffled
    (positions mapped by the index pass): identical answers up to the shuffle, and both against
    the brute force on a sample; duplicates appended at the end break the order (general path)."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(11 + kind)
    L = 16
    wl2 = synthetic.whitelist_codes(60_000, L, seed=5 + kind)  # sorted: alphabetical
    wl = wl2 if kind == 2 else synthetic.two_to_three(wl2, L)
    q = wl[rng.integers(0, wl.size, 200_000)].copy()
    pos = rng.integers(0, L, q.size).astype(np.uint64)
    w = np.uint64(kind)
    sub = rng.integers(0, 4, q.size).astype(np.uint64) + (np.uint64(1) if kind == 3 else np.uint64(0))
    m = rng.random(q.size)
    one = m < 0.5
    q[one] = (q[one] & ~(np.uint64((1 << kind) - 1) << (w * pos[one]))) | (sub[one] << (w * pos[one]))
    if kind == 3:
        nn = (m >= 0.5) & (m < 0.65)
        q[nn] = q[nn] & ~(np.uint64(7) << (w * pos[nn]))  # N
    perm = rng.permutation(wl.size)
    out = {}
    for name, w_ in (("sorted", wl), ("shuffled", wl[perm]), ("dups", np.concatenate([wl, wl[:3]]))):
        d_wl = torch.from_numpy(np.ascontiguousarray(w_).view(np.int64)).cuda()
        d_q = torch.from_numpy(q.view(np.int64)).cuda()
        plan = _lib.NearestPlan(kind, d_wl.data_ptr(), w_.size, kind * L, 1)
        assert plan.info()["scheme"] == "halves"
        oi = torch.empty(q.size, dtype=torch.int32, device="cuda")
        od = torch.empty(q.size, dtype=torch.uint8, device="cuda")
        plan.query(d_q.data_ptr(), q.size, oi.data_ptr(), od.data_ptr())
        torch.cuda.synchronize()
        plan.close()
        out[name] = (oi.cpu().numpy(), od.cpu().numpy())
    si, sd = out["sorted"]
    hi, hd = out["shuffled"]
    mapped = np.where(hi >= 0, perm[np.maximum(hi, 0)], hi)
    assert np.array_equal(mapped, si) and np.array_equal(hd, sd)
    samp = rng.integers(0, q.size, 4000)
    ridx, rdist = O.c_nearest(kind, wl, q[samp], 1)
    assert np.array_equal(si[samp], ridx) and np.array_equal(sd[samp], rdist)
    # with the duplicates (ties at distance 0 and 1 with their first copies) against the brute force
    di, dd = out["dups"]
    ridx, rdist = O.c_nearest(kind, np.concatenate([wl, wl[:3]]), q[samp], 1)
    assert np.array_equal(di[samp], ridx) and np.array_equal(dd[samp], rdist)
    near_dups = np.isin(q, wl[:3])
    assert (di[near_dups] == -2).all()


@pytest.mark.parametrize("kind", [2, 3])
@pytest.mark.parametrize("order", ["ACGT", "ACTG", "CAGT", "TGCA"])
@pytest.mark.parametrize("L", [16, 13])
def test_nearest_halves_whitelist_orders(kind, order, L):
    """Whitelists sorted in each candidate digit order of the half-key build (alphabetical as a
    10x file, TwoBit-numeric, ThreeBit-numeric) and in one that is none of them (reverse
    alphabetical: the general path), at an even and an odd length: the brute force's answers,
    max_d 0 and 1, ties from one duplicated code included."""
    rng = np.random.default_rng(1000 * kind + 10 * L + ["ACGT", "ACTG", "CAGT", "TGCA"].index(order))
    wl2 = synthetic.whitelist_codes(20_000, L, seed=L + kind)
    seqs = synthetic.decode_ascii(wl2, L)
    rank = np.zeros(256, dtype=np.int64)
    for i, ch in enumerate(order.encode()):
        rank[ch] = i
    keys = rank[seqs]
    srt = np.lexsort(keys.T[::-1])  # lexicographic in `order`'s digit ranks, first base most significant
    wl2 = wl2[srt]
    wl2 = np.insert(wl2, 5000, wl2[5000])  # one duplicated code, kept in order
    wl = wl2 if kind == 2 else synthetic.two_to_three(wl2, L)
    q = wl[rng.integers(0, wl.size, 3000)].copy()
    pos = rng.integers(0, L, q.size).astype(np.uint64)
    w = np.uint64(kind)
    sub = rng.integers(0, 4, q.size).astype(np.uint64) + (np.uint64(1) if kind == 3 else np.uint64(0))
    one = rng.random(q.size) < 0.6
    q[one] = (q[one] & ~(np.uint64((1 << kind) - 1) << (w * pos[one]))) | (sub[one] << (w * pos[one]))
    for max_d in (0, 1):
        idx, dist = barcode.nearest_whitelist(q, wl, max_distance=max_d, encoding=kind)
        ridx, rdist = O.c_nearest(kind, wl, q, max_d)
        assert np.array_equal(idx, ridx) and np.array_equal(dist, rdist), (order, max_d)


@pytest.mark.parametrize("kind,max_d", [(3, 1), (2, 1), (3, 0), (3, 2), (2, 2)])
def test_whitelist_corrector_batches(kind, max_d):
    """WhitelistCorrector (one device index, many host batches) against nearest_whitelist and
    the brute force: several batches, an empty one, a page-locked one; the caller's whitelist
    changed after construction changes nothing; an empty whitelist finds nothing."""
    rng = np.random.default_rng(90 + 10 * kind + max_d)
    L = 16
    wl2 = synthetic.whitelist_codes(6000, L, seed=31 + kind)
    wl = wl2 if kind == 2 else synthetic.two_to_three(wl2, L)
    wl = np.concatenate([wl, wl[:5]])  # duplicates: ties
    keep = wl.copy()
    corr = barcode.WhitelistCorrector(wl, max_distance=max_d, encoding=kind)
    wl[:] = 0  # (the corrector holds its own copy)
    batches = []
    for size in (5000, 0, 1, 12345):
        q = keep[rng.integers(0, keep.size, size)]
        pos = rng.integers(0, L, size).astype(np.uint64)
        one = rng.random(size) < 0.5
        w = np.uint64(kind)
        sub = rng.integers(0, 4, size).astype(np.uint64) + (np.uint64(1) if kind == 3 else np.uint64(0))
        q[one] = (q[one] & ~(np.uint64((1 << kind) - 1) << (w * pos[one]))) | (sub[one] << (w * pos[one]))
        batches.append(q)
    pin = _lib.pinned.empty(batches[3].size, np.uint64)
    pin[:] = batches[3]
    batches.append(pin)
    for q in batches:
        idx, dist = corr.nearest(q)
        ridx, rdist = O.c_nearest(kind, keep, q, max_d)
        assert np.array_equal(idx, ridx) and np.array_equal(dist, rdist)
        idx2, dist2 = barcode.nearest_whitelist(q, keep, max_distance=max_d, encoding=kind)
        assert np.array_equal(idx, idx2) and np.array_equal(dist, dist2)
    # a flow-piece-sized batch (1.1M queries), page-locked and pageable: equal to the same
    # queries sent as smaller batches, and to the brute force on a sample
    big = batches[0][rng.integers(0, batches[0].size, 1_100_003)]
    parts = [corr.nearest(big[s:s + 300_000]) for s in range(0, big.size, 300_000)]
    pidx, pdist = np.concatenate([p[0] for p in parts]), np.concatenate([p[1] for p in parts])
    bigp = _lib.pinned.empty(big.size, np.uint64)
    bigp[:] = big
    samp = rng.integers(0, big.size, 3000)
    ridx, rdist = O.c_nearest(kind, keep, big[samp], max_d)
    for q in (big, bigp):
        idx, dist = corr.nearest(q)
        assert np.array_equal(idx, pidx) and np.array_equal(dist, pdist)
        assert np.array_equal(idx[samp], ridx) and np.array_equal(dist[samp], rdist)
    corr.close()
    empty = barcode.WhitelistCorrector(np.zeros(0, np.uint64), max_distance=max_d, encoding=kind)
    idx, dist = empty.nearest(batches[0][:10])
    assert (idx == -1).all() and (dist == 255).all()


def test_nearest_halves_falls_back_on_non_acgt_whitelists():
    """A ThreeBit whitelist holding an N (or a shorter code) cannot use the half-key tables:
    the plan takes another layout and the result is still the brute force's."""
    import torch
    wl = synthetic.two_to_three(synthetic.whitelist_codes(3000, 16, seed=9), 16)
    wl[5] = (wl[5] & ~np.uint64(7)) | np.uint64(6)   # an N
    wl[6] = wl[6] >> np.uint64(3)                    # a 15-base code
    q = np.concatenate([wl[:500], wl[500:1000] ^ np.uint64(3 << 9)])
    d_wl = torch.from_numpy(wl.view(np.int64)).cuda()
    plan = _lib.NearestPlan(3, d_wl.data_ptr(), wl.size, 48, 1)
    assert plan.info()["scheme"] != "halves"
    plan.close()
    idx, dist = barcode.nearest_whitelist(q, wl, max_distance=1, encoding=3)
    ridx, rdist = O.c_nearest(3, wl, q, 1)
    assert np.array_equal(idx, ridx) and np.array_equal(dist, rdist)


def _nearest_vs_bruteforce(kind, max_d):
    rng = np.random.default_rng(100 + 10 * kind + max_d)
    wl_codes2 = synthetic.whitelist_codes(3000, 16, seed=kind * 7 + max_d)
    wl_seqs = synthetic.decode_ascii(wl_codes2, 16)
    q_seqs = _config4_queries(wl_seqs, 4000, rng, b"ACGT" if kind == 3 else b"ACGT")
    if kind == 2:
        q_seqs[q_seqs == ord("N")] = ord("A")
    enc = ThreeBit if kind == 3 else TwoBit
    wl = enc.encode_array(wl_seqs)
    q = enc.encode_array(q_seqs)
    idx, dist = barcode.nearest_whitelist(q, wl, max_distance=max_d, encoding=kind)
    ridx, rdist = O.nearest_bruteforce(kind, wl, q, max_d)
    assert np.array_equal(idx, ridx)
    assert np.array_equal(dist, rdist)


def test_nearest_ties_and_edges():
    # two whitelist codes at distance 2; the midpoint query is at distance 1 from both
    a = ThreeBit.encode(b"ACGTACGTACGTACGT")
    b = ThreeBit.encode(b"ACGTACGTACGTACTA")
    mid = ThreeBit.encode(b"ACGTACGTACGTACTT")
    wl = np.array([a, b], dtype=np.uint64)
    idx, dist = barcode.nearest_whitelist([mid, a, b, ThreeBit.encode(b"N" * 16)], wl, 1)
    assert idx.tolist() == [-2, 0, 1, -1]
    assert dist.tolist() == [1, 0, 0, 255]
    # duplicated whitelist entries are distinct indices -> tie
    idx, dist = barcode.nearest_whitelist([a], np.array([a, a], dtype=np.uint64), 0)
    assert idx.tolist() == [-2] and dist.tolist() == [0]
    # empty inputs
    idx, dist = barcode.nearest_whitelist([], wl, 1)
    assert idx.size == 0
    idx, dist = barcode.nearest_whitelist([a], np.array([], dtype=np.uint64), 1)
    assert idx.tolist() == [-1]


def test_barcodes_nearest_method(golden):
    rec = golden["nearest"]["two"]
    s = barcode.PriorBarcodeSet.from_iterable_encoded([int(c) for c in rec["whitelist"]], 16)
    idx, dist = s.nearest(np.array([int(c) for c in rec["queries"]], dtype=np.uint64), 1)
    assert idx.tolist() == rec["result"]["1"]["index"]


def test_allpairs_counter_flush_path():
    # force the in-kernel u32 -> u64 counter flush after every work-queue pull
    codes = synthetic.whitelist_codes(9000, 16, seed=21)
    with _lib.tuning(allpairs_flush_items=1, allpairs_grab=3):
        hist = _lib.hamming_hist_allpairs(codes, 32)
    assert hist.astype(np.int64).tolist() == O.c_hist_rows(codes)[:17].tolist()


@pytest.mark.parametrize("L", [4, 15, 16, 21, 28, 32])
def test_encode_tiled_matches_bytewise(L):
    rng = np.random.default_rng(L)
    n = 100_003
    seqs = np.frombuffer(b"ACGTacgt", np.uint8)[rng.integers(0, 8, (n, L))]
    for enc, ref in ((TwoBit, O.two_bit_encode), (ThreeBit, O.three_bit_encode)):
        if enc is ThreeBit and L > 21:
            continue
        codes, gc = enc.encode_array(seqs, return_gc=True)
        for r in list(range(0, n, 997)) + [n - 1]:
            s = seqs[r].tobytes()
            assert int(codes[r]) == ref(s)
            assert int(gc[r]) == s.upper().count(b"C") + s.upper().count(b"G")


def test_from_whitelist_line_semantics(golden, tmp_path):
    for rec in golden["from_whitelist"]:
        p = tmp_path / (rec["name"] + ".txt")
        p.write_bytes(bytes.fromhex(rec["content"]))
        random.seed(11)
        if "error" in rec:
            with pytest.raises(KeyError) as ei:
                barcode.Barcodes.from_whitelist(str(p), 16)
            assert list(ei.value.args) == rec["error"]["args"], rec["name"]
        else:
            b = barcode.Barcodes.from_whitelist(str(p), 16)
            assert [str(k) for k in b] == rec["codes"], rec["name"]
            assert [b[k] for k in b] == rec["counts"], rec["name"]
        assert random.getrandbits(32) == rec["after"], rec["name"]


def test_encode_stream_pipeline():
    rng = np.random.default_rng(55)
    n, L = 3_000_017, 28
    seqs = np.frombuffer(b"ACGTacgtN", np.uint8)[rng.integers(0, 9, (n, L))]
    codes, gc, flags = _lib.encode_stream(2, seqs, chunk=700_001)
    c2, g2, f2 = _lib.encode(2, seqs[:200_000], L)
    assert np.array_equal(codes[:200_000], c2[:, 0]) and np.array_equal(gc[:200_000], g2)
    assert np.array_equal(flags[:200_000], f2)
    for r in range(0, n, 99_991):
        s = seqs[r].tobytes()
        if b"N" not in s:
            assert int(codes[r]) == O.two_bit_encode(s)
            assert flags[r] == 0
        else:
            assert flags[r] == 1
    # the drop-in batch path routes >= 1M records through the stream
    random.seed(3)
    a = TwoBit.encode_array(seqs[:1_100_000])
    random.seed(3)
    b = [TwoBit.encode(seqs[r].tobytes()) for r in range(0, 1000)]
    assert a[:1000].tolist() == b


# ---------------------------------------------------------------- headline sizes vs the oracle
def test_pinned_pool_blocks_reused_after_last_view():
    """_lib.pinned: arrays over page-locked blocks (DMA in place); a block goes back to the pool
    only when the last view of its array is freed, and the next array of its size class reuses it."""
    import gc as _gc
    pool = _lib.PinnedPool(keep_bytes=64 << 20)
    a = pool.empty((3 << 20,), np.uint8)
    assert _lib.host_pinned(a)
    p0 = a.ctypes.data
    a[:] = 7
    v = a[1000:2000]
    del a
    _gc.collect()
    b = pool.empty(3 << 20, np.uint8)
    assert b.ctypes.data != p0  # the view still holds the first block
    assert int(v.sum()) == 7 * 1000
    del v
    _gc.collect()
    c = pool.empty((2 << 20, 2), np.uint8)  # same 4 MiB class: the first block again
    assert c.ctypes.data == p0 and _lib.host_pinned(c)
    small = pool.empty(100, np.int32)  # below MIN_BYTES: plain numpy
    assert small.shape == (100,) and not _lib.host_pinned(small)
    del b, c
    _gc.collect()
    pool.trim()
    assert pool._idle == 0 and not pool._free and pool._held == 0
    capped = _lib.PinnedPool(keep_bytes=0, max_bytes=4 << 20)  # one 4 MiB block at a time
    x = capped.empty(3 << 20, np.uint8)
    y = capped.empty(3 << 20, np.uint8)  # over the cap: plain numpy
    assert _lib.host_pinned(x) and not _lib.host_pinned(y)
    del x
    _gc.collect()
    assert capped._held == 0  # (keep_bytes = 0: freed at once)
    z = capped.empty(3 << 20, np.uint8)
    assert _lib.host_pinned(z)


def test_encode_stream_pinned_and_pageable():
    """The host stream copies page-locked buffers in place and pageable ones through its own pinned
    stage (it never registers caller memory): both give the same codes, GC and flags, for inputs
    and outputs pinned or not, a view into a larger block, and ranges that run past a pinned block."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(57)
    n, L = 2_500_003, 16
    seqs = np.frombuffer(b"ACGTN", np.uint8)[rng.integers(0, 5, (n, L))]
    want = _lib.encode_stream(2, seqs, chunk=1 << 20)
    assert not _lib.host_pinned(seqs)
    pin = torch.empty((n + 5, L), dtype=torch.uint8, pin_memory=True).numpy()
    pin[:n] = seqs
    assert _lib.host_pinned(pin) and _lib.host_pinned(pin[3:n])
    big = torch.empty((n + 5) * L + 4096, dtype=torch.uint8, pin_memory=True).numpy()
    base = big.ctypes.data
    assert _lib.host_pinned(big)
    # a range that starts inside the block and runs past its end (1 TiB) is not in place
    import ctypes
    out = ctypes.c_int(7)
    _lib.check(_lib.lib().sct_host_pinned(ctypes.c_void_p(base + 64), 1 << 40, ctypes.byref(out)))
    assert out.value == 0
    codes = torch.empty(n, dtype=torch.int64, pin_memory=True).numpy().view(np.uint64)
    gc = torch.empty(n, dtype=torch.uint8, pin_memory=True).numpy()
    fl = torch.empty(n, dtype=torch.uint8, pin_memory=True).numpy()
    f = _lib.lib().sct_encode_stream_host
    for src in (pin[:n], seqs):
        for outs in ((codes, gc, fl), tuple(np.zeros_like(a) for a in (codes, gc, fl))):
            for a in outs:
                a[:] = 0
            _lib.check(f(2, _lib._ptr(src), n, L, _lib._ptr(outs[0]), _lib._ptr(outs[1]), _lib._ptr(outs[2]), 0))
            for a, b in zip(outs, want):
                assert np.array_equal(a, b)
    # a pinned input view that is not at its block's start; a one-record and a two-chunk stream
    got = _lib.encode_stream(2, pin[3:n], chunk=1 << 19)
    for a, b in zip(got, want):
        assert np.array_equal(a, b[3:])
    one = _lib.encode_stream(2, seqs[:1])
    assert int(one[0][0]) == int(want[0][0])


def test_allpairs_737k_spectral_bin_for_bin():
    """Config 2 at full size: AUTO (= SPECTRAL) histogram of all 271,790,530,560 pairs,
    bin for bin against the C oracle's AVX-512 popcount loop over every pair."""
    n, L, seed = synthetic.CONFIGS[2]
    codes = synthetic.whitelist_codes(n, L, seed)
    torch = pytest.importorskip("torch")
    d_codes = torch.from_numpy(codes.view(np.int64)).cuda()
    plan = _lib.AllPairsPlan(d_codes.data_ptr(), n, 32)
    assert plan.scheme == _lib.SCHEME_SPECTRAL
    plan.close()
    hist = sharding.allpairs_histogram_sharded(codes, 32)
    ref, simd = O.c_hist16(codes)
    assert hist.astype(np.int64).tolist() == ref[:17].tolist()
    assert int(hist.sum()) == n * (n - 1) // 2
    # the drop-in on the same set
    s = barcode.Barcodes.from_iterable_encoded(codes.tolist(), 16)
    assert s.summarize_hamming_distances() == O.summary_from_hist_numpy(ref[:17])


@pytest.mark.parametrize("m", [126, 127, 128, 129])
def test_allpairs_spectral_column_width_edges(m):
    """A transform column (low 14 bits) holding exactly m codes: 127 is the last int8
    intermediate, 128 the first int16; 128 / 129 are the last 4-group / first 5-group
    column of the plane build.  SPECTRAL vs the oracle."""
    rng = np.random.default_rng(m)
    hi = np.unique(rng.integers(0, 1 << 18, 4 * m).astype(np.uint64))[:m]
    col = (hi << np.uint64(14)) | np.uint64(0x1ABC)
    rest = synthetic.whitelist_codes(5000, 16, seed=m)
    rest = rest[(rest & np.uint64(0x3FFF)) != np.uint64(0x1ABC)]
    codes = np.concatenate([col, rest])
    rng.shuffle(codes)
    assert np.bincount((codes & np.uint64(0x3FFF)).astype(np.int64)).max() == m
    hist = _spectral_hist(codes, [(0, 1 << 17), (1 << 17, 1 << 18)])
    assert hist.astype(np.int64).tolist() == O.c_hist16(codes)[0][:17].tolist()


@pytest.mark.parametrize("case", ["m127", "m97", "m65", "ragged"])
def test_allpairs_spectral_seed_group_counts(case):
    """The int8 seed's step-major walk against the C oracle for every group count: a column
    of 127 codes (a fourth group from L2), 97 (the first fourth group), 65 (three groups in
    registers) beside columns of one or two groups, and slice ranges that cut walks."""
    m = {"m127": 127, "m97": 97, "m65": 65, "ragged": 40}[case]
    rng = np.random.default_rng(m)
    hi = np.unique(rng.integers(0, 1 << 18, 4 * m).astype(np.uint64))[:m]
    col = (hi << np.uint64(14)) | np.uint64(0x2345)
    rest = synthetic.whitelist_codes(7000, 16, seed=m)
    rest = rest[(rest & np.uint64(0x3FFF)) != np.uint64(0x2345)]
    codes = np.concatenate([col, rest])
    ranges = [(0, 1 << 18)] if case != "ragged" else [(0, 1001), (1001, 70001), (70001, 1 << 18)]
    hist = _spectral_hist(codes, ranges)
    assert hist.astype(np.int64).tolist() == O.c_hist16(codes)[0][:17].tolist()


def _dense_columns(splits, n_rand, seed):
    """n_rand random 16-bp codes plus, per entry of `splits`, one 14-bit column holding
    sum(split) codes (> 127: int16 seeds on 14-bit columns) spread over its four 16-bit
    sub-columns as `split` (each <= 127)."""
    rng = np.random.default_rng(seed)
    parts, used = [], set()
    for j, split in enumerate(splits):
        col = int(rng.integers(0, 1 << 14))
        while col in used:
            col = int(rng.integers(0, 1 << 14))
        used.add(col)
        for s, k in enumerate(split):  # sub-column s: bits 14, 15 = s
            hi = rng.choice(1 << 16, k, replace=False).astype(np.uint64)
            parts.append((hi << np.uint64(16)) | np.uint64((s << 14) | col))
    rest = synthetic.whitelist_codes(n_rand, 16, seed=seed)
    rest = rest[~np.isin((rest & np.uint64(0x3FFF)).astype(np.int64), list(used))]
    codes = np.concatenate(parts + [rest])
    rng.shuffle(codes)
    return codes


@pytest.mark.parametrize("case", ["two_columns", "sub127", "ragged", "small_chunk"])
def test_allpairs_spectral_16bit_columns(case):
    """Sets whose densest 14-bit column needs int16 seeds but whose 16-bit columns hold <= 127
    codes take the 16-bit-column transform (spectral16.hip): bin for bin against the C oracle.
    Sub-columns of 127 (four groups, the int8 limit), 65 (the first third group), 0 and 1
    codes; slice ranges cutting walks and chunks; a small chunk (several seed / tile passes
    and their digit-weight orders)."""
    torch = pytest.importorskip("torch")
    splits = {"two_columns": [(40, 40, 40, 40), (100, 0, 1, 60)], "sub127": [(127, 65, 0, 3)],
              "ragged": [(90, 90, 0, 0)], "small_chunk": [(33, 64, 96, 127)]}[case]
    codes = _dense_columns(splits, 6000, seed=len(case))
    ranges = [(0, 1 << 18)]
    chunk = None
    if case == "ragged":
        ranges = [(0, 1001), (1001, 70001), (70001, 1 << 18)]
    if case == "small_chunk":
        chunk, ranges = 4096, [(0, 8192), (8192, 100000), (100000, 1 << 18)]
    d_codes = torch.from_numpy(codes.view(np.int64)).cuda()
    with _lib.tuning(spectral_chunk=chunk):
        plan = _lib.AllPairsPlan(d_codes.data_ptr(), codes.size, 32, scheme=_lib.SCHEME_SPECTRAL)
    info = plan.spectral_info()
    plan.close()
    assert info["column_bits"] == 16 and info["elem_bytes"] == 1 and info["max_column"] <= 127
    hist = _spectral_hist(codes, ranges, chunk=chunk)
    assert hist.astype(np.int64).tolist() == O.c_hist16(codes)[0][:17].tolist()


def test_allpairs_spectral_16bit_not_taken():
    """A 16-bit column of 128 codes: no int8 layout fits, so the plan keeps 14-bit columns with
    int16 seeds (and stays exact)."""
    torch = pytest.importorskip("torch")
    codes = _dense_columns([(128, 10, 10, 10)], 3000, seed=9)
    d_codes = torch.from_numpy(codes.view(np.int64)).cuda()
    plan = _lib.AllPairsPlan(d_codes.data_ptr(), codes.size, 32, scheme=_lib.SCHEME_SPECTRAL)
    info = plan.spectral_info()
    plan.close()
    assert info["column_bits"] == 14 and info["elem_bytes"] == 2
    hist = _spectral_hist(codes)
    assert hist.astype(np.int64).tolist() == O.c_hist16(codes)[0][:17].tolist()


def test_allpairs_config5_spectral_bin_for_bin():
    """Config 5's 3,686,400 codes (int16 intermediate, ~225 codes per column): AUTO (=
    SPECTRAL) bin for bin against the C oracle's count of all 6,794,770,636,800 pairs
    (barcode.py:39-46; ~20 s on the box's 16 cores), and against the pair-enumerating MOMENTS
    kernel and the mean distance the per-position base counts imply."""
    torch = pytest.importorskip("torch")
    n, L, seed = synthetic.CONFIGS[5]
    codes = synthetic.whitelist_codes(n, L, seed)
    d_codes = torch.from_numpy(codes.view(np.int64)).cuda()
    plan = _lib.AllPairsPlan(d_codes.data_ptr(), n, 32)
    assert plan.scheme == _lib.SCHEME_SPECTRAL
    assert plan.spectral_info()["column_bits"] == 16  # int8 seeds on 16-bit columns
    plan.close()
    hs = sharding.allpairs_histogram_sharded(d_codes, 32)
    ref, _ = O.c_hist16(codes)
    assert hs.astype(np.int64).tolist() == ref[:17].tolist()
    hm = sharding.allpairs_histogram_sharded(d_codes, 32, scheme=_lib.SCHEME_MOMENTS)
    assert hs.tolist() == hm.tolist()
    P = n * (n - 1) // 2
    assert int(hs.sum()) == P
    bases = (codes[:, None] >> (2 * np.arange(16, dtype=np.uint64))) & np.uint64(3)
    agree = 0
    for p in range(16):
        cnt = np.bincount(bases[:, p].astype(np.int64), minlength=4).astype(object)
        agree += int(cnt.dot(cnt - 1)) // 2
    assert sum(d * int(x) for d, x in enumerate(hs)) == 16 * P - agree


def test_encode_config5_1e9_reads_device_resident():
    """Config 5's read stream at full size: 1e9 random 28-bp reads generated on the device
    (1 % with one N), TwoBit-encoded with GC on the device (sct_encode, encodings.py:75-88,
    102-111) in two record ranges, as two ranks would.  Every code, GC count and flag is
    checked against values computed independently from the generating bases (torch, on the
    device); every 10^6-th record also against the oracle's statement-for-statement encoder."""
    torch = pytest.importorskip("torch")
    n, L = synthetic.CONFIG5_READS, synthetic.CONFIG5_READ_LENGTH
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(5)
    b = torch.randint(0, 4, (n, L), dtype=torch.uint8, device=dev, generator=g)  # TwoBit values A0 C1 T2 G3
    seqs = torch.empty_like(b)
    chunk = 50_000_000
    for r0 in range(0, n, chunk):  # ASCII: A 65, C 67, T 84, G 71
        x = b[r0:r0 + chunk]
        seqs[r0:r0 + chunk] = 65 + 2 * x + 15 * (x == 2).to(torch.uint8)
    nrows = torch.arange(0, n, 100, device=dev)  # 1 % of the reads get one N
    npos = torch.randint(0, L, (nrows.numel(),), device=dev, generator=g)
    seqs[nrows, npos] = ord("N")
    codes = torch.empty(n, dtype=torch.int64, device=dev)
    gc = torch.empty(n, dtype=torch.uint8, device=dev)
    flags = torch.empty(n, dtype=torch.uint8, device=dev)
    lib = _lib.lib()
    for r0, r1 in ((0, n // 2), (n // 2, n)):
        _lib.check(lib.sct_encode(2, seqs[r0].data_ptr(), r1 - r0, L, L, codes[r0].data_ptr(), gc[r0].data_ptr(),
                                  flags[r0].data_ptr(), None))
    torch.cuda.synchronize()
    isn = torch.zeros(n, dtype=torch.bool, device=dev)
    isn[nrows] = True
    bad = 0
    gc_total = 0
    for r0 in range(0, n, chunk):
        x = b[r0:r0 + chunk]
        nm = isn[r0:r0 + chunk]
        want = torch.zeros(x.shape[0], dtype=torch.int64, device=dev)
        wgc = torch.zeros(x.shape[0], dtype=torch.int32, device=dev)
        for i in range(L):
            v = x[:, i].to(torch.int64)
            want = (want << 2) | v
            wgc += (v & 1).to(torch.int32)
        # the N read: that base encodes as 0, is not GC, and flags the record (bit 0)
        k = nrows[(nrows >= r0) & (nrows < r0 + x.shape[0])]
        kp = npos[(nrows >= r0) & (nrows < r0 + x.shape[0])]
        vk = b[k, kp].to(torch.int64)
        want[k - r0] &= ~(vk << (2 * (L - 1 - kp)))
        wgc[k - r0] -= (vk & 1).to(torch.int32)
        bad += int((codes[r0:r0 + chunk] != want).sum())
        bad += int((gc[r0:r0 + chunk].to(torch.int32) != wgc).sum())
        bad += int((flags[r0:r0 + chunk] != nm.to(torch.uint8)).sum())
        gc_total += int(gc[r0:r0 + chunk].to(torch.int64).sum())
    assert bad == 0
    want_gc = sum(int((seqs[r0:r0 + chunk] == ord("C")).sum()) + int((seqs[r0:r0 + chunk] == ord("G")).sum())
                  for r0 in range(0, n, chunk))
    assert gc_total == want_gc
    for r in range(7, n, 1_000_000):  # (every 100th read holds an N: these hold none)
        s = bytes(seqs[r].cpu().numpy().tobytes())
        assert b"N" not in s
        assert int(codes[r]) == O.two_bit_encode(s) and int(flags[r]) == 0
        assert int(gc[r]) == s.count(b"C") + s.count(b"G")


# ---------------------------------------------------------------- keys >= 2^64 (multi-limb)
def test_wide_sets_golden(golden_wide):
    """ThreeBit-encoded 22..28-bp whitelists, TwoBit > 32 bp and mixed-width key sets
    through the drop-in: the reference's own summaries and histograms."""
    for rec in golden_wide:
        s = barcode.Barcodes.from_iterable_encoded([int(c) for c in rec["codes"]], rec["L"])
        if "error" in rec:
            with pytest.raises(IndexError):
                s.summarize_hamming_distances()
            continue
        assert s.summarize_hamming_distances() == fromhex(rec["summary"]), (rec["kind"], rec["L"])
        h = s.hamming_histogram()
        nz = len(rec["hist"])
        assert h[:nz].astype(np.int64).tolist() == rec["hist"] and not h[nz:].any()


@pytest.mark.parametrize("words,n", [(1, 3000), (2, 20_000), (2, 257), (3, 4097), (4, 3000), (5, 1000), (9, 600)])
def test_wide_kernel_vs_oracle(words, n):
    """Every limb count the wide kernel specialises (1-4 private-counter columns, 5+ the
    shared-histogram path) against the C oracle, with duplicates and near neighbours."""
    rng = np.random.default_rng(words * 1000 + n)
    limbs = rng.integers(0, 2 ** 63, size=(n, words), dtype=np.uint64) * np.uint64(2) + \
        rng.integers(0, 2, size=(n, words), dtype=np.uint64)
    limbs[n // 2:n // 2 + 10] = limbs[:10]  # duplicates (d = 0)
    limbs[n // 3, -1] ^= np.uint64(1 << 40)  # a near neighbour of row n/3 + 1
    limbs[n // 3 + 1] = limbs[n // 3]
    limbs[n // 3 + 1, -1] ^= np.uint64(3 << 20)
    hist = _lib.hamming_hist_allpairs_wide(limbs)
    ref = O.c_hist_wide(limbs)
    assert hist.astype(np.int64).tolist() == ref.tolist()
    assert int(hist.sum()) == n * (n - 1) // 2


def test_wide_kernel_item_ranges_sum_to_whole():
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(8)
    n, words = 5000, 2
    limbs = rng.integers(0, 2 ** 62, size=(n, words), dtype=np.uint64)
    items, nb = _lib.wide_geometry(n, words)
    d = torch.from_numpy(limbs.view(np.int64)).cuda()
    total = torch.zeros(nb, dtype=torch.int64, device="cuda")
    cuts = [0, 1, items // 5, items // 2 + 3, items - 1, items]
    pairs = 0
    for b, e in zip(cuts[:-1], cuts[1:]):
        _lib.check(_lib.lib().sct_allpairs_wide(d.data_ptr(), n, words, b, e, total.data_ptr(), nb, None))
        pairs += _lib.wide_range_pairs(n, b, e)
    torch.cuda.synchronize()
    assert pairs == n * (n - 1) // 2
    assert total.cpu().numpy().tolist() == O.c_hist_wide(limbs).tolist()


# ---------------------------------------------------------------- config 4 at full size
@pytest.mark.parametrize("scheme", ["auto", "oa"])
def test_nearest_config4_full_size(scheme):
    """Config 4 as specified: the 737,280-code ThreeBit whitelist and 100M observed
    barcodes (50 % exact, 25 % substitution, 15 % N, 10 % random) at max_d = 1.  Every
    exact draw must come back as its own index at distance 0, every one-edit query within
    distance 1; 20,000 sampled queries of every class bit-exact against the OpenMP brute
    force over the whole whitelist.  AUTO = the half-key tables (L2-resident); OA = the
    open-addressing pair-key tables."""
    torch = pytest.importorskip("torch")
    n, L, seed = synthetic.CONFIGS[4]
    wl = synthetic.two_to_three(synthetic.whitelist_codes(n, L, seed), L)
    nq = 100_000_000
    q, pick, cls = synthetic.config4_queries(wl, nq, seed=4)
    d_wl = torch.from_numpy(wl.view(np.int64)).cuda()
    idx = torch.empty(nq, dtype=torch.int32, device="cuda")
    dist = torch.empty(nq, dtype=torch.uint8, device="cuda")
    with _lib.tuning(nearest_scheme=_NEAREST_SCHEMES[scheme]):
        plan = _lib.NearestPlan(3, d_wl.data_ptr(), n, 3 * L, 1)
    plan.query(q.data_ptr(), nq, idx.data_ptr(), dist.data_ptr())
    torch.cuda.synchronize()
    plan.close()
    exact = cls == 0
    assert torch.equal(idx[exact].long(), pick[exact]) and bool((dist[exact] == 0).all())
    one = (cls == 1) | (cls == 2)
    assert bool((dist[one] <= 1).all()) and bool((idx[one] != -1).all())
    g = torch.Generator(device="cuda").manual_seed(44)
    samp = torch.randint(0, nq, (20_000,), device="cuda", generator=g)
    ridx, rdist = O.c_nearest(3, wl, q[samp].cpu().numpy().view(np.uint64), 1)
    assert np.array_equal(idx[samp].cpu().numpy(), ridx)
    assert np.array_equal(dist[samp].cpu().numpy(), rdist)
    # the drop-in entry point on the sampled queries
    i2, d2 = barcode.nearest_whitelist(q[samp].cpu().numpy().view(np.uint64), wl, 1)
    assert np.array_equal(i2, ridx) and np.array_equal(d2, rdist)


@pytest.mark.parametrize("kind,max_d", [(2, 7), (3, 7), (2, 5)])
def test_nearest_max_d_near_limit(kind, max_d):
    """max_d + 1 = 8 / 6 blocks of 2-3 bases: block values shared by thousands of codes
    (buckets of ~nw / 16 entries) -- the duplicate flagging sorts instead of scanning pairs."""
    rng = np.random.default_rng(70 + kind + max_d)
    wl2 = synthetic.whitelist_codes(20_000, 16, seed=kind + max_d)
    wl = wl2 if kind == 2 else synthetic.two_to_three(wl2)
    wl = np.concatenate([wl, wl[:25]])  # duplicates -> ties
    q = np.concatenate([wl[:500], rng.permutation(wl)[:500] ^ np.uint64(1 << 5)])
    idx, dist = barcode.nearest_whitelist(q, wl, max_distance=max_d, encoding=kind)
    ridx, rdist = O.c_nearest(kind, wl, q, max_d)
    assert np.array_equal(idx, ridx) and np.array_equal(dist, rdist)


@pytest.mark.parametrize("scheme", [0, 1, 2])
@pytest.mark.parametrize("build_on", ["side", "main"])
def test_sharded_run_pipelined_steps_match_oracle(scheme, build_on):
    """ShardedAllPairs.run (what bench.py times): steps pipelined two deep over two count
    buffers, the build beside the previous count or in line; every step's histogram equals
    step()'s and the oracle's (barcode.py:39-46)."""
    n = 6_000 if scheme == 0 else 20_000
    codes = synthetic.whitelist_codes(n, 16, 77 + scheme)
    ref = O.c_hist16(codes)[0][:17].tolist()
    with sharding.ShardedAllPairs(codes, 32, scheme) as job:
        job.build_on = build_on
        assert job.step().tolist() == ref
        for steps in (1, 2, 5):
            hists = job.run(steps, timing=True)
            assert len(hists) == steps and all(h.tolist() == ref for h in hists)
        assert job.step().tolist() == ref


def test_all_negative_keys_summary():
    """An all-negative key set through the drop-in (barcode.py:39-46: the reference's
    ``a ^ b`` of two negatives is non-negative and its loop counts it): the summary of the
    reference's own pair loop, restated (oracle.two_bit_hamming, encodings.py:113-121)."""
    rng = np.random.default_rng(17)
    keys = [-int(v) for v in rng.integers(1, 1 << 32, 300)] + [-(2 ** 40) - 3, -1]
    keys = list(dict.fromkeys(keys))
    d = [O.two_bit_hamming(a, b) for a, b in itertools.combinations(keys, 2)]
    s = barcode.Barcodes.from_iterable_encoded(keys, 16)
    assert s.summarize_hamming_distances() == O.summary_numpy(d)


# ---------------------------------------------------------------- one-limb variable-length encode, base_frequency
@pytest.mark.parametrize("kind", [2, 3])
@pytest.mark.parametrize("layout", ["lines", "scattered"])
def test_encode_var_one_limb(kind, layout):
    """sct_encode_var with one limb (encode_var_kernel): consecutive lines (staged through
    LDS) and records scattered over a 4 MB buffer (the global-memory branch), with empty,
    ambiguous and invalid records, vs oracle.two_bit_encode / three_bit_encode and the GC
    bits (encodings.py:75-88, 102-111, 155-167, 182-192)."""
    import torch
    rng = np.random.default_rng(31 + kind)
    maxL = 32 if kind == 2 else 21
    n = 70_001
    lens = rng.integers(0, maxL + 1, n).astype(np.int32)
    alphabet = np.frombuffer(b"ACGTacgt", np.uint8)
    recs = [alphabet[rng.integers(0, 8, L)].tobytes() for L in lens]
    for i in rng.choice(n, 300, replace=False):
        if lens[i]:
            b = bytearray(recs[i])
            b[rng.integers(0, lens[i])] = rng.choice(list(b"NRx#\r"))
            recs[i] = bytes(b)
    if layout == "lines":
        data = b"".join(r + b"\n" for r in recs)
        starts = np.cumsum([0] + [len(r) + 1 for r in recs[:-1]]).astype(np.int64)
    else:
        size = 4 << 20
        buf = bytearray(rng.integers(0, 256, size, dtype=np.uint8).tobytes())
        starts = rng.integers(0, size - maxL, n).astype(np.int64)
        for s, r in zip(starts, recs):  # later records may overwrite earlier ones' bytes
            buf[s:s + len(r)] = r
        recs = [bytes(buf[s:s + L]) for s, L in zip(starts, lens)]
        data = bytes(buf)
    dev = torch.device("cuda", 0)
    d_buf = torch.from_numpy(np.frombuffer(data, np.uint8).copy()).to(dev)
    d_st = torch.from_numpy(starts).to(dev)
    d_len = torch.from_numpy(lens).to(dev)
    codes = torch.empty(n, dtype=torch.int64, device=dev)
    gc = torch.empty(n, dtype=torch.uint8, device=dev)
    flags = torch.empty(n, dtype=torch.uint8, device=dev)
    _lib.check(_lib.lib().sct_encode_var(kind, d_buf.data_ptr(), d_st.data_ptr(), d_len.data_ptr(), n, 1,
                                         codes.data_ptr(), gc.data_ptr(), flags.data_ptr(), None))
    torch.cuda.synchronize()
    got = codes.cpu().numpy().view(np.uint64)
    g, f = gc.cpu().numpy(), flags.cpu().numpy()
    for i, r in enumerate(recs):
        if kind == 3:
            want = O.three_bit_encode(r)
            assert (int(got[i]), int(g[i]), int(f[i])) == (want, O.three_bit_gc(want), 0), i
            continue
        amb = any(c in b"NRnr" for c in r)
        bad = any(c not in b"ACGTacgtNRnr" for c in r)
        assert int(f[i]) == (1 if amb else 0) | (2 if bad else 0), i
        if not (amb or bad):
            want = O.two_bit_encode(r)
            assert (int(got[i]), int(g[i])) == (want, O.two_bit_gc(want, len(r))), i


@pytest.mark.parametrize("L", [1, 7, 16, 31, 32, 33, 40])
def test_base_frequency_lengths(L):
    """base_frequency_kernel (ballot counts of the 2-bit fields) vs oracle.base_frequency_numpy
    (barcode.py:48-70) for lengths around the 64-bit key width, ragged n, and n = 0, 1."""
    rng = np.random.default_rng(L)
    bits = min(2 * L, 64)
    for n in (0, 1, 63, 65, 100_003):
        codes = rng.integers(0, 1 << 62, n, dtype=np.uint64) * np.uint64(4) + rng.integers(0, 4, n, dtype=np.uint64)
        if bits < 64:
            codes &= np.uint64((1 << bits) - 1)
        got = _lib.base_frequency(codes, L)
        want = O.base_frequency_numpy(codes, L)
        assert np.array_equal(got, want), (L, n)


@pytest.mark.parametrize("L", [1, 5, 12, 16])
def test_base_frequency_short_codes(L):
    """The 32-bit form (L <= 16: base_frequency16_kernel) vs oracle.base_frequency_numpy: bits
    above 2L set (never read), one and two rounds of 15 codes per lane, ragged n; and the byte
    counters at their bound: a constant code repeated so that lanes see exactly 255 codes."""
    rng = np.random.default_rng(100 + L)
    for n in (15 * 256 * 7 + 3, 3_000_017) + ((20_000_003,) if L == 16 else ()):
        codes = rng.integers(0, 1 << 63, n, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, n, dtype=np.uint64)
        assert np.array_equal(_lib.base_frequency(codes, L), O.base_frequency_numpy(codes, L)), (L, n)
    if L == 16:
        n = 4096 * 255 * 256 + 1  # the grid's 255-codes-per-lane bound
        c = 0xDEADBEEF00000000 | 0b11100100_01001110_10110001_00011011
        got = _lib.base_frequency(np.full(n, c, np.uint64), L)
        want = np.zeros((L, 4), np.uint64)
        for p in range(L):
            want[p, (c >> (2 * (L - 1 - p))) & 3] = n
        assert np.array_equal(got.reshape(L, 4), want)


def test_lines_capacity_short_fills_nothing():
    """sct_lines with room for fewer lines than the buffer holds reports the count, a longest
    line of 0 and leaves the outputs untouched; with room for all of them it fills them
    (barcode.py:96-97: every line's [:-1])."""
    import ctypes

    import torch
    data = b"ACGT\nAC\n\nGGGGG\nT"
    d_buf = torch.tensor(list(data), dtype=torch.uint8, device="cuda")
    lib = _lib.lib()
    for cap in (4, 5, 9):
        starts = torch.full((9,), -7, dtype=torch.int64, device="cuda")
        lens = torch.full((9,), -7, dtype=torch.int32, device="cuda")
        nl, mx = ctypes.c_int64(0), ctypes.c_int32(0)
        _lib.check(lib.sct_lines(d_buf.data_ptr(), len(data), cap, starts.data_ptr(), lens.data_ptr(),
                                 ctypes.byref(nl), ctypes.byref(mx), None))
        assert nl.value == 5
        if cap < 5:
            assert mx.value == 0 and (starts == -7).all() and (lens == -7).all()
        else:
            lines = data.split(b"\n")
            want_len = [len(x) for x in lines[:-1]] + [len(lines[-1]) - 1]
            assert lens[:5].tolist() == want_len and mx.value == max(want_len)
            assert starts[:5].tolist() == [0, 5, 8, 9, 15]
            assert (starts[5:] == -7).all()


def _ref_lines(data):
    """(start, chopped length) of every line as barcode.py:95-97 iterates a binary file:
    lines end at '\\n' (included), a last line may lack it, `line[:-1]` drops the last byte."""
    out, pos = [], 0
    while pos < len(data):
        e = data.find(b"\n", pos)
        e = len(data) - 1 if e < 0 else e
        out.append((pos, e - pos))
        pos = e + 1
    return out


def _ingest_cases():
    rng = np.random.default_rng(404)
    alpha = np.frombuffer(b"ACGTacgtNRY", dtype=np.uint8)
    cases = {"tiny": b"ACGT\nAC\n\nGGGGG\nT", "crlf": b"ACGTACGT\r\nGGCC\r\n", "empty_lines": b"\n\n\nA\n",
             "no_final_lf": b"ACGTTGCA\nACG", "single_byte": b"A", "only_lf": b"\n"}
    parts = []  # ragged lines: 0-40 bytes (TwoBit > 32 bases: two limbs; flag 4 at words = 1)
    for k in range(30_000):
        L = int(rng.integers(0, 41)) if k % 97 else int(rng.integers(200, 9000))  # some lines span tiles
        parts.append(alpha[rng.integers(0, alpha.size, L)].tobytes() + b"\n")
    parts.append(b"X" * 20_000)  # a final line of 20 KB without '\n': tiles with no line end at all
    cases["ragged"] = b"".join(parts)
    # upper-case A/C/G/T only (the SWAR path, no LUT fallback): every length 0-40 at every
    # alignment, lines crossing the 4 KiB sub-tiles and 16 KiB tiles, a few N lines among them
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    parts = []
    for k in range(60_000):
        L = k % 41 if k % 211 else int(rng.integers(100, 3000))
        rec = acgt[rng.integers(0, 4, L)].tobytes()
        if k % 1009 == 5 and L:
            rec = rec[:L // 2] + b"N" + rec[L // 2 + 1:]
        parts.append(rec + b"\n")
    cases["acgt"] = b"".join(parts)
    # fixed-stride files (the encode pass numbers lines by arithmetic): 16 / 32 / 21 bases, empty
    # lines, a stride-4 file whose last line has no '\n' (its last base is chopped, as the
    # reference's line[:-1]), N and lower-case lines among them, and one line end off the stride
    # in a 340 KB file (every other tile fixed: the file must take the general path)
    for L in (16, 32, 21):
        recs = [acgt[rng.integers(0, 4, L)].tobytes() for _ in range(20_000 if L == 16 else 8_000)]
        recs[7] = b"N" + recs[7][1:]
        recs[11] = recs[11].lower()
        cases["fixed%d" % L] = b"\n".join(recs) + b"\n"
    cases["fixed_empty"] = b"\n" * 20_000
    cases["fixed_no_final_lf"] = b"ACG\n" * 10_000 + b"TGCA"
    odd = bytearray(b"ACGTACGTACGTACGT\n" * 20_000)
    odd[170_000:170_017] = b"ACGTACGTACGTACG\nA"  # one end moved by one byte
    cases["fixed_one_off"] = bytes(odd)
    # sizes that are multiples of 17 with a 17-byte first line, but not 16-base lines throughout: the
    # one-read pass (whitelist_spec16_kernel) must notice and leave the file to the general path
    split = bytearray(b"ACGTACGTACGTACGT\n" * 20_000)
    split[85_000:85_017] = b"ACGTACG\nACGTACGT\n"  # two lines in one 17-byte slot (an inner '\n')
    cases["fixed_split_line"] = bytes(split)
    cases["fixed_long_line"] = b"ACGTACGTACGTACGT\n" * 9_000 + b"ACGT" * 8 + b"A\n" + b"TTTTGGGGCCCCAAAA\n" * 9_000
    return cases


@pytest.mark.parametrize("name", list(_ingest_cases()))
@pytest.mark.parametrize("kind,words", [(2, 1), (2, 2), (3, 1), (3, 2)])
def test_whitelist_encode_one_pass(name, kind, words):
    _whitelist_encode_check(name, kind, words)


@pytest.mark.parametrize("name", ["ragged", "acgt", "fixed16", "fixed_one_off"])
def test_whitelist_encode_with_reduction_launch(name):
    """The same with the tile prefixes from the coarse sums of tile_sums_reduce_kernel (the form
    buffers above 64 MiB take), not summed by every encode workgroup."""
    with _lib.tuning(ingest_direct=0):
        _whitelist_encode_check(name, 2, 1)


@pytest.mark.parametrize("name", ["fixed16", "fixed_one_off", "fixed_split_line", "tiny"])
def test_whitelist_encode_without_one_read(name):
    """The count + encode passes on their own (SCT_TUNE_INGEST_SPEC = 0): the 16-base fixed-stride
    branch of the encode pass, which the one-read pass otherwise takes over."""
    with _lib.tuning(ingest_spec=0):
        _whitelist_encode_check(name, 2, 1)
        _whitelist_encode_check(name, 3, 1)


def _whitelist_encode_check(name, kind, words):
    """sct_whitelist_encode (count pass, tile-sum reduction, encode pass; asynchronous) against
    the reference's binary line loop with `line[:-1]` (barcode.py:95-97) and the oracle's
    encoders (encodings.py:75-88 / 155-167): line count, longest line, every start, length,
    code limb, GC count and flag; lines too long for `words` limbs carry flag 4; a capacity
    below the count writes only the lines below it."""
    import torch
    data = _ingest_cases()[name]
    ref = _ref_lines(data)
    n = len(ref)
    d_buf = torch.tensor(list(data), dtype=torch.uint8, device="cuda")
    lib = _lib.lib()
    for cap in (n, max(0, n - 3)):
        codes = torch.full((max(1, n) * words,), -5, dtype=torch.int64, device="cuda")
        starts = torch.full((max(1, n),), -5, dtype=torch.int64, device="cuda")
        lens = torch.full((max(1, n),), -5, dtype=torch.int32, device="cuda")
        gc = torch.zeros(max(1, n), dtype=torch.uint8, device="cuda")
        flags = torch.full((max(1, n),), 77, dtype=torch.uint8, device="cuda")
        d_n = torch.full((1,), -1, dtype=torch.int64, device="cuda")
        d_mx = torch.full((1,), -1, dtype=torch.int32, device="cuda")
        _lib.check(lib.sct_whitelist_encode(d_buf.data_ptr(), len(data), kind, words, cap, codes.data_ptr(),
                                            starts.data_ptr(), lens.data_ptr(), gc.data_ptr(), flags.data_ptr(),
                                            d_n.data_ptr(), d_mx.data_ptr(), None))
        torch.cuda.synchronize()
        assert int(d_n.item()) == n and int(d_mx.item()) == max([L for _, L in ref], default=0)
        st, ln = starts.cpu().numpy(), lens.cpu().numpy()
        cd = codes.cpu().numpy().view(np.uint64).reshape(-1, words)
        fl, g = flags.cpu().numpy(), gc.cpu().numpy()
        assert st[:cap].tolist() == [s for s, _ in ref[:cap]] and ln[:cap].tolist() == [L for _, L in ref[:cap]]
        assert (st[cap:n] == -5).all() and (fl[cap:n] == 77).all()
        enc = O.two_bit_encode if kind == 2 else O.three_bit_encode
        for i, (s0, L) in enumerate(ref[:cap]):
            rec = data[s0:s0 + L]
            if kind * L > 64 * words:
                assert fl[i] == 4
                continue
            amb = kind == 2 and any(b in b"MRWSYKVHDBNmrwsykvhdbn" for b in rec)
            bad = kind == 2 and any(b not in b"ACGTacgtMRWSYKVHDBNmrwsykvhdbn" for b in rec)
            assert fl[i] == (1 if amb else 0) | (2 if bad else 0), (i, rec)
            if amb or bad:
                continue
            want = enc(rec)
            assert _lib.limbs_to_ints(cd[i:i + 1])[0] == want, (i, rec)
            gcw = rec.upper().count(b"C") + rec.upper().count(b"G")
            assert g[i] == min(255, gcw)
