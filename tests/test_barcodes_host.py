"""CPU: host-side semantics of sctools_amd.barcode.Barcodes that need no kernel -- the
key array is rebuilt from the mapping on every call (no stale cache), non-integer keys
raise the reference's own TypeError from `a ^ b` (encodings.py:117 via barcode.py:42-43),
keys >= 2^64 become multi-limb rows."""

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
    with pytest.raises(ValueError):
        barcode.Barcodes({-1: 1, 2 ** 65: 1}, 4).codes_array()
    with pytest.raises(OverflowError):  # as the reference's np.fromiter (barcode.py:59)
        b.base_frequency()


def test_base4_entropy_golden(golden):
    """stats.base4_entropy on the reference's own base counts reproduces the
    effective_diversity the reference computed from them, bit for bit."""
    from sctools_amd.stats import base4_entropy
    wl = golden["whitelist_1k"]
    got = base4_entropy(np.array(wl["base_frequency"]))
    assert [float(v) for v in got] == [float.fromhex(v) for v in wl["effective_diversity"]]
