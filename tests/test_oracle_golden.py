"""CPU: pin the oracle (oracle/oracle.py, oracle/sct_oracle.c) against the golden
fixtures generated from the reference itself (tests/golden/gen_golden.py)."""

import itertools
import random

import numpy as np
import pytest

from conftest import fromhex
from oracle import oracle as O
from sctools_amd import _lib, synthetic


def test_encode(golden):
    for rec in golden["encode"]:
        seq = bytes.fromhex(rec["seq"])
        fn = O.two_bit_encode if rec["enc"] == 2 else O.three_bit_encode
        if "error" in rec:
            with pytest.raises(KeyError) as ei:
                fn(seq)
            assert list(ei.value.args) == rec["error"]["args"]
        else:
            assert fn(seq) == int(rec["code"])


def test_encode_ambiguous_rng(golden):
    for case in golden["encode_ambiguous"]:
        random.seed(case["seed"])
        got = []
        try:
            for s in case["seqs"]:
                got.append(str(O.two_bit_encode(bytes.fromhex(s))))
        except KeyError as e:
            assert case.get("error") and list(e.args) == case["error"]["args"]
        assert got == case["codes"]
        assert random.getrandbits(32) == case["after"]


def test_decode_gc(golden):
    for rec in golden["decode2"]:
        code = int(rec["code"])
        assert O.two_bit_decode(code, rec["L"]) == bytes.fromhex(rec["decoded"])
        assert O.two_bit_gc(code, rec["L"]) == rec["gc"]
    for rec in golden["decode3"]:
        code = int(rec["code"])
        assert O.three_bit_gc(code) == rec["gc"]
        if "error" in rec:
            with pytest.raises(KeyError) as ei:
                O.three_bit_decode(code)
            assert list(ei.value.args) == rec["error"]["args"]
        else:
            assert O.three_bit_decode(code) == bytes.fromhex(rec["decoded"])


def test_hamming(golden):
    for a, b, d2, d3 in golden["hamming"]:
        assert O.two_bit_hamming(int(a), int(b)) == d2
        assert O.three_bit_hamming(int(a), int(b)) == d3
    rows = [r for r in golden["hamming"] if int(r[0]) < 2 ** 64 and int(r[1]) < 2 ** 64]
    a = np.array([int(r[0]) for r in rows], dtype=np.uint64)
    b = np.array([int(r[1]) for r in rows], dtype=np.uint64)
    assert O.pair_distances_numpy(a, b).tolist() == [r[2] for r in rows]


def test_simple_barcodes(golden):
    sb = golden["simple_barcodes"]
    seqs = [bytes.fromhex(s) for s in sb["seqs"]]
    two = [O.two_bit_hamming(O.two_bit_encode(a), O.two_bit_encode(b)) for a, b in itertools.combinations(seqs, 2)]
    assert two == sb["two"]


def test_whitelist_hist_and_summary(golden):
    wl = golden["whitelist_1k"]
    codes = np.array([int(c) for c in wl["codes"]], dtype=np.uint64)
    assert O.allpairs_hist_numpy(codes, 17).tolist() == wl["hist"]
    assert O.c_hist_rows(codes)[:17].tolist() == wl["hist"]
    assert O.c_hist_rows(codes, scalar=True)[:17].tolist() == wl["hist"]
    assert O.summary_from_hist_numpy(wl["hist"]) == fromhex(wl["summary"])
    assert O.base_frequency_numpy(codes, 16).tolist() == wl["base_frequency"]


def test_small_sets_summary(golden):
    for rec in golden["small_sets"]:
        keys = list(dict.fromkeys(int(c) for c in rec["codes"]))
        dists = [O.two_bit_hamming(a, b) for a, b in itertools.combinations(keys, 2)]
        if rec["error"]:
            with pytest.raises(IndexError):
                O.summary_numpy(dists)
            continue
        want = fromhex(rec["summary"])
        assert {k: float(v) for k, v in O.summary_numpy(dists).items()} == want
        hist = np.bincount(dists, minlength=65)
        assert O.summary_from_hist_numpy(hist) == want


def test_config1_10k(golden_10k):
    codes = synthetic.whitelist_codes(golden_10k["n"], golden_10k["L"], golden_10k["seed"])
    assert [str(int(c)) for c in codes[:8]] == golden_10k["codes_sha_first"]
    hist = O.c_hist_rows(codes)[:17]
    assert hist.tolist() == golden_10k["hist"]
    assert O.summary_from_hist_numpy(hist) == fromhex(golden_10k["summary"])


def test_item_enumeration_covers_all_pairs():
    codes = synthetic.whitelist_codes(3000, 16, seed=4)
    lib = O.c_oracle()
    ref = O.c_hist_rows(codes)
    hist = np.zeros(65, dtype=np.int64)
    pairs = np.zeros(1, dtype=np.int64)
    lib.oracle_hist_items(codes.ctypes.data, codes.size, 256, 1024, hist.ctypes.data, 0, 1 << 40,
                          pairs.ctypes.data, 1)
    assert int(pairs[0]) == 3000 * 2999 // 2
    assert hist.tolist() == ref.tolist()


def test_nearest_bruteforce(golden):
    for name, kind in (("three", 3), ("two", 2)):
        rec = golden["nearest"][name]
        wl = [int(c) for c in rec["whitelist"]]
        q = [int(c) for c in rec["queries"]]
        for md, want in rec["result"].items():
            idx, dist = O.nearest_bruteforce(kind, wl, q, int(md))
            assert idx.tolist() == want["index"]
            assert dist.tolist() == want["dist"]


def test_c_hist16_pinned(golden, golden_10k):
    """The AVX-512 checker of every full-size all-pairs parity test (config 2, 4, 5, the
    multisets) against the reference's own histograms: whole sets, row ranges, threads."""
    wl = golden["whitelist_1k"]
    codes = np.array([int(c) for c in wl["codes"]], dtype=np.uint64)
    hist, _ = O.c_hist16(codes)
    assert hist[:17].tolist() == wl["hist"] and not hist[17:].any()
    parts = sum(O.c_hist16(codes, b, e, threads=t)[0] for b, e, t in ((0, 1, 1), (1, 333, 2), (333, 1000, 0)))
    assert parts[:17].tolist() == wl["hist"]
    c10 = synthetic.whitelist_codes(golden_10k["n"], golden_10k["L"], golden_10k["seed"])
    hist, simd = O.c_hist16(c10)
    assert hist[:17].tolist() == golden_10k["hist"] and not hist[17:].any()
    # duplicates (the multiset tests): d = 0 pairs against the scalar restatement
    dup = np.concatenate([c10[:3000], c10[:500], c10[:1]])
    assert O.c_hist16(dup)[0].tolist() == O.c_hist_rows(dup, scalar=True).tolist()


def test_c_nearest_pinned(golden):
    """The OpenMP checker of the config-4 / FASTQ nearest tests against the reference's own
    distances (golden["nearest"], composed from TwoBit/ThreeBit.hamming_distance)."""
    for name, kind in (("three", 3), ("two", 2)):
        rec = golden["nearest"][name]
        wl = np.array([int(c) for c in rec["whitelist"]], dtype=np.uint64)
        q = np.array([int(c) for c in rec["queries"]], dtype=np.uint64)
        for md, want in rec["result"].items():
            for threads in (1, 0):
                idx, dist = O.c_nearest(kind, wl, q, int(md), threads=threads)
                assert idx.tolist() == want["index"]
                assert dist.tolist() == want["dist"]


def test_negative_ints_oracle(golden_edges):
    """The oracle's digit loops on negative ints against the reference's (edges.json)."""
    for rec in golden_edges["twobit_negative"]:
        x, L = int(rec["code"]), rec["L"]
        assert O.two_bit_decode(x, L).hex() == rec["decode"]["bytes"]
        assert O.two_bit_gc(x, L) == int(rec["gc"]["value"])
    for a, b, d2, d3 in golden_edges["hamming_negative"]:
        assert O.two_bit_hamming(int(a), int(b)) == d2
        assert O.three_bit_hamming(int(a), int(b)) == d3
    for rec in golden_edges["threebit_decode_negative"]:
        with pytest.raises(KeyError) as ei:
            O.three_bit_decode(int(rec["code"]))
        assert list(ei.value.args) == rec["decode"]["error"]["args"]


def test_from_whitelist_semantics_oracle(golden):
    from collections import Counter
    for rec in golden["from_whitelist"]:
        lines = bytes.fromhex(rec["content"]).splitlines(keepends=True)
        random.seed(11)
        try:
            c = Counter(O.two_bit_encode(ln[:-1]) for ln in lines)
            assert "error" not in rec
            assert [str(k) for k in c] == rec["codes"] and list(c.values()) == rec["counts"]
        except KeyError as e:
            assert list(e.args) == rec["error"]["args"]
        assert random.getrandbits(32) == rec["after"]


# ---------------------------------------------------------------- MOMENTS scheme identities
def test_moments_identity_on_reference_histograms(golden, golden_10k):
    """The agreement moments counted from position marginals (what the MOMENTS scheme's
    moments pass computes) equal sum_d hist[d] C(16-d, k) on the reference's own golden
    histograms, and the 17 MOMENTS counts of those histograms invert exactly through
    the library's host solver (no GPU)."""
    wl = golden["whitelist_1k"]
    codes = np.array([int(c) for c in wl["codes"]], dtype=np.uint64)
    assert O.moments_from_marginals(codes) == O.moments_from_hist(wl["hist"])
    assert _lib.counts_to_hist(O.moment_counts_from_hist(wl["hist"]), _lib.SCHEME_MOMENTS,
                               17).tolist() == wl["hist"]
    c10 = synthetic.whitelist_codes(golden_10k["n"], golden_10k["L"], golden_10k["seed"])
    h10 = golden_10k["hist"]
    assert O.moments_from_marginals(c10) == O.moments_from_hist(h10)
    assert _lib.counts_to_hist(O.moment_counts_from_hist(h10), _lib.SCHEME_MOMENTS,
                               17).tolist() == list(h10)


def test_moments_solver_rejects_inconsistent_counts():
    c = O.moment_counts_from_hist([0, 3, 5, 0, 0, 7, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 1])
    c[14] += 1  # M_1 off by one: no integral histogram
    with pytest.raises(ValueError):
        _lib.counts_to_hist(c, _lib.SCHEME_MOMENTS, 17)


# ---------------------------------------------------------------- SPECTRAL scheme identities
def _pair_hist_digits(codes, G):
    h = [0] * (G + 1)
    for a, b in itertools.combinations([int(c) for c in codes], 2):
        x = a ^ b
        h[sum(1 for i in range(G) if (x >> (2 * i)) & 3)] += 1
    return h


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_spectral_identity_small_space(seed):
    """The SPECTRAL scheme's algebra, checked with an explicit Walsh-Hadamard transform in a
    space small enough for numpy (G = 5 bases, 2^10 points): S_w = sum over z with w
    non-zero digits of F(z)^2, then N(d) = 2^-2G sum_w S_w K_d(w) and (N(d) - n[d=0]) / 2
    equal the brute-force pair histogram (duplicates included)."""
    G = 5
    rng = np.random.default_rng(seed)
    codes = rng.integers(0, 1 << (2 * G), 60 + 20 * seed)
    codes = np.concatenate([codes, codes[:7]])  # duplicates: d = 0 pairs
    f = np.bincount(codes, minlength=1 << (2 * G)).astype(np.int64)
    H = np.array([[1]])
    for _ in range(2 * G):
        H = np.block([[H, H], [H, -H]])
    F = H @ f
    z = np.arange(1 << (2 * G))
    wt = np.array([sum(1 for i in range(G) if (int(v) >> (2 * i)) & 3) for v in z])
    S = [int((F[wt == w] ** 2).sum()) for w in range(G + 1)]
    K = O.krawtchouk4(G)
    n = codes.size
    got = []
    for d in range(G + 1):
        N = sum(S[w] * K[d][w] for w in range(G + 1))
        assert N % (1 << (2 * G)) == 0
        N //= 1 << (2 * G)
        got.append((N - (n if d == 0 else 0)) // 2)
    assert got == _pair_hist_digits(codes, G)
    # and the forward map the tests use gives the same S
    assert O.spectral_weight_sums(got, n) == S
    c = O.spectral_counts_from_hist(got, n)
    assert c[0] == n and int(c[1]) == 2 * got[0] + n
    W = G + 1
    assert [int(c[2 + w]) + (int(c[2 + W + w]) << 32) + (int(c[2 + 2 * W + w]) << 64) for w in range(W)] == S


def test_spectral_counts_invert_on_reference_histograms(golden, golden_10k):
    """The 18 SPECTRAL counts of the reference's golden histograms invert exactly through
    the library's host Krawtchouk transform (no GPU)."""
    wl = golden["whitelist_1k"]
    n1 = len(wl["codes"])
    assert _lib.counts_to_hist(O.spectral_counts_from_hist(wl["hist"], n1),
                               _lib.SCHEME_SPECTRAL).tolist() == wl["hist"]
    h10 = golden_10k["hist"]
    assert _lib.counts_to_hist(O.spectral_counts_from_hist(h10, golden_10k["n"]),
                               _lib.SCHEME_SPECTRAL, 17).tolist() == list(h10)


def test_spectral_rejects_inconsistent_counts():
    hist = [0, 0, 0, 1, 0, 2, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0]  # 3 codes
    c = O.spectral_counts_from_hist(hist, 3)
    assert _lib.counts_to_hist(c, _lib.SCHEME_SPECTRAL).tolist() == hist
    # S_2 + 1; n + 1 (S_0 != n^2); S_15 + 2^32; sum f^2 + 1; S_3 + 2^64 (what a 2^64 wrap of one
    # weight sum would do: every Krawtchouk bin stays integral and even, only the check
    # sum_w S_w == 2^32 sum f^2 sees it)
    for i, delta in ((4, 1), (0, 1), (17, 1 << 32), (1, 1), (39, 1)):
        bad = c.copy()
        bad[i] += np.uint64(delta)
        with pytest.raises(ValueError):
            _lib.counts_to_hist(bad, _lib.SCHEME_SPECTRAL)


def test_geometry_picks_spectral_for_large_whitelists():
    """Host-only: AUTO resolves to SPECTRAL at 16 bases from 325K codes (the measured
    crossover; SCT_TUNE_SPECTRAL_MIN_N moves it): the 2^18 transform slices are the work items."""
    assert _lib.allpairs_geometry(3_700_000, 32)["items"] == 1 << 18
    assert _lib.allpairs_geometry(737_280, 32)["items"] == 1 << 18
    assert _lib.allpairs_geometry(400_000, 32)["items"] == 1 << 18
    assert _lib.allpairs_geometry(300_000, 32)["items"] != 1 << 18
    assert _lib.allpairs_geometry(3_700_000, 40)["items"] != 1 << 18  # 20 bases: SUBSETS


def test_wide_sets_oracle(golden_wide):
    """Keys >= 2^64 (ThreeBit 22..28 bp, TwoBit > 32 bp, mixed widths): the multi-limb C
    oracle and the histogram summary against the reference's own numbers."""
    for rec in golden_wide:
        codes = list(dict.fromkeys(int(c) for c in rec["codes"]))  # Counter keys, insertion order
        words = _lib.words_for_bits(max(c.bit_length() for c in codes))
        hist = O.c_hist_wide(_lib.ints_to_limbs(codes, words))
        nz = len(rec["hist"])
        assert hist[:nz].tolist() == rec["hist"] and not hist[nz:].any()
        if "summary" in rec:
            assert O.summary_from_hist_numpy(rec["hist"]) == fromhex(rec["summary"])
        else:
            assert len(codes) < 2
