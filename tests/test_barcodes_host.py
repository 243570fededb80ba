"""CPU: host-side semantics of sctools_amd.barcode.Barcodes that need no kernel -- the
key array is rebuilt from the mapping on every call (no stale cache), non-integer keys
raise the reference's own TypeError from `a ^ b` (encodings.py:117 via barcode.py:42-43),
keys >= 2^64 become multi-limb rows, all-negative keys keep their pairwise XORs."""

import numpy as np
import pytest

from sctools_amd import barcode


def test_codes_follow_in_place_mutation():
    d = {5: 1, 9: 2, 12: 1}
    b = barcode.Barcodes(d, 4)
    assert b.codes_array().tolist() == [5, 9, 12]
    del d[9]
    d[77] = 3  # same length, different key
    assert b.codes_array().tolist() == [5, 12, 77]


@pytest.mark.parametrize("bad", [2.5, "ACGT", b"AC", None])
def test_non_integer_keys_raise_the_references_type_error(bad):
    b = barcode.Barcodes({3: 1, bad: 1, 4: 1}, 4)
    with pytest.raises(TypeError) as ei:
        b.summarize_hamming_distances()
    with pytest.raises(TypeError) as ref:
        3 ^ bad  # what barcode.py:42-43 -> encodings.py:117 evaluates first
    assert str(ei.value) == str(ref.value)


def test_wide_and_negative_keys():
    b = barcode.Barcodes({1: 1, 2 ** 70 + 3: 1, 2 ** 64: 1}, 40)
    arr = b.codes_array()
    assert arr.shape == (3, 2) and arr.dtype == np.uint64
    assert arr.tolist() == [[1, 0], [3, 64], [0, 1]]
    with pytest.raises(ValueError):  # mixed signs: the reference's loop never ends
        barcode.Barcodes({-1: 1, 2 ** 65: 1}, 4).codes_array()
    with pytest.raises(ValueError):
        barcode.Barcodes({-5: 1, 7: 2}, 4).codes_array()
    assert barcode.Barcodes({-5: 1}, 4).codes_array().size == 1  # one key: no pair, no XOR
    with pytest.raises(OverflowError):  # as the reference's np.fromiter (barcode.py:59)
        b.base_frequency()


@pytest.mark.parametrize("keys", [
    [-1, -2, -3, -4, -1000, -(2 ** 31)],
    [-(2 ** 63), -1, -(2 ** 40) + 7, -12345],
    [-(2 ** 70), -(2 ** 70) + 5, -3, -(2 ** 66) - 1],
])
def test_all_negative_keys_keep_every_pairwise_xor(keys):
    """All-negative key sets (barcode.py:39-46 runs on them: a ^ b of two negatives is
    non-negative): the kernel codes keep every pairwise XOR, so every distance, exactly."""
    from oracle import oracle as O
    from sctools_amd import _lib
    arr = barcode.Barcodes({k: 1 for k in keys}, 16).codes_array()
    vals = arr.tolist() if arr.ndim == 1 else _lib.limbs_to_ints(arr)
    for i in range(len(keys)):
        for j in range(i + 1, len(keys)):
            assert vals[i] ^ vals[j] == keys[i] ^ keys[j]
            assert O.two_bit_hamming(vals[i], vals[j]) == O.two_bit_hamming(keys[i], keys[j])


@pytest.mark.parametrize("keys", [[-3, -7, -12], [-(2 ** 70), -5], [-1]])
def test_nearest_rejects_negative_keys(keys):
    """Barcodes.nearest compares the set's codes with OUTSIDE queries, where the pairwise
    masking of all-negative keys would give plausible but wrong matches: any
    negative key raises ValueError before a device call, while the pairwise codes of the
    same set stay available to the summary."""
    b = barcode.Barcodes({k: 1 for k in keys}, 16)
    with pytest.raises(ValueError, match="non-negative"):
        b.nearest(np.array([0, 5], dtype=np.uint64))
    assert len(b.codes_array()) == len(keys)


def test_base4_entropy_golden(golden):
    """stats.base4_entropy on the reference's own base counts reproduces the
    effective_diversity the reference computed from them, bit for bit."""
    from sctools_amd.stats import base4_entropy
    wl = golden["whitelist_1k"]
    got = base4_entropy(np.array(wl["base_frequency"]))
    assert [float(v) for v in got] == [float.fromhex(v) for v in wl["effective_diversity"]]


def _keys_seq(keys):
    """The key loop's contract (csrc/pykeys.c) restated in Python: (status, count, min, max)."""
    out, lo, hi = [], None, None
    for k in keys:
        if not isinstance(k, int):
            return 1, len(out), lo, hi
        if not -(1 << 63) <= k < (1 << 63):
            return 2, len(out), lo, hi
        out.append(int(k))
        lo = k if lo is None else min(lo, k)
        hi = k if hi is None else max(hi, k)
    return 0, len(out), lo, hi


@pytest.mark.parametrize("case", ["plain", "negative", "bool_and_limits", "str_late", "float_early", "big_mid",
                                  "deleted", "counter"])
def test_parallel_key_loop_matches_sequential(case):
    """Dicts of >= 2^17 keys take the threaded key loop (csrc/pykeys.c, four runs of the
    entries array): the same keys, order, min / max, and the same stop status and count as
    the sequential contract, wherever in the runs a non-int or a too-wide int sits."""
    from collections import Counter

    from sctools_amd import _pykeys
    rng = np.random.default_rng(7)
    n = 300_001
    keys = [int(v) for v in rng.integers(0, 1 << 62, n)]
    if case == "negative":
        keys = [-k for k in keys]
    elif case == "bool_and_limits":
        keys[0], keys[1], keys[n // 2], keys[-1] = True, False, (1 << 63) - 1, -(1 << 63) + 1
    elif case == "str_late":
        keys[n - 5] = "ACGT"
    elif case == "float_early":
        keys[3] = 1.5
    elif case == "big_mid":
        keys[n // 4 + 3] = 1 << 70
    keys = list(dict.fromkeys(keys))  # (unique, insertion order)
    d = Counter(dict.fromkeys(keys, 1)) if case == "counter" else dict.fromkeys(keys, 1)
    if case == "deleted":
        for k in keys[10:20]:
            del d[k]
        keys = keys[:10] + keys[20:]
    arr = np.zeros(len(keys), np.int64)
    status, count, lo, hi = _pykeys.keys_to_int64(d, arr)
    want = _keys_seq(keys)
    assert (status, count) == want[:2]
    assert arr[:count].tolist() == [int(k) for k in keys[:count]]
    if status == 0:
        assert (lo, hi) == want[2:]
