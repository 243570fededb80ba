"""CPU: the C-ABI library loads and exports every symbol include/sctools_hip.h
declares, and its host-only logic (Moebius inversion, numpy-exact summary) is
right.  No kernel is launched here (there is no GPU in the build container)."""

import os
import re

import numpy as np
import pytest

from conftest import ROOT, fromhex
from oracle import oracle as O
from sctools_amd import _lib


def header_symbols():
    with open(os.path.join(ROOT, "include", "sctools_hip.h")) as f:
        text = f.read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(sct_\w+)\s*\(", text, re.M)))


def test_library_exports_header_symbols():
    lib = _lib.lib()
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
    # and the ctypes signature table covers exactly the header
    assert sorted(_lib.SIGNATURES) == syms


def test_version_and_errors():
    lib = _lib.lib()
    assert lib.sct_version() == 1
    rc = lib.sct_counts_to_hist(None, 3, None)
    assert rc == _lib.SCT_E_INVALID
    assert "NULL" in _lib.last_error()


def test_compute_without_gpu_fails_loudly():
    if _lib.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(RuntimeError):
        _lib.hamming_hist_allpairs(np.arange(10, dtype=np.uint64))


def subset_counts(hist):
    hist = np.asarray(hist, dtype=np.uint64)
    counts = np.zeros_like(hist)
    for m in range(hist.size):
        counts[m] = sum(int(hist[d]) for d in range(hist.size) if (d & m) == m)
    return counts


@pytest.mark.parametrize("nbins", [2, 3, 5, 9, 13, 17, 25, 33, 65])
def test_counts_to_hist_inverts(nbins):
    rng = np.random.default_rng(nbins)
    for _ in range(20):
        hist = rng.integers(0, 10 ** 11, size=nbins).astype(np.uint64)
        hist[rng.random(nbins) < 0.3] = 0
        assert _lib.counts_to_hist(subset_counts(hist)).tolist() == hist.tolist()


def test_counts_to_hist_rejects_inconsistent():
    with pytest.raises(ValueError):
        _lib.counts_to_hist(np.array([1, 5, 0], dtype=np.uint64))


def test_summary_from_hist_golden(golden):
    wl = golden["whitelist_1k"]
    vals = _lib.summary_from_hist(np.array(wl["hist"], dtype=np.uint64))
    want = fromhex(wl["summary"])
    assert vals.tolist() == list(want.values())
    for rec in golden["small_sets"]:
        if rec["error"]:
            continue
        keys = list(dict.fromkeys(int(c) for c in rec["codes"]))
        hist = np.zeros(65, dtype=np.uint64)
        for i in range(len(keys)):
            for j in range(i + 1, len(keys)):
                hist[O.two_bit_hamming(keys[i], keys[j])] += 1
        assert _lib.summary_from_hist(hist).tolist() == list(fromhex(rec["summary"]).values())


def test_summary_matches_numpy_random():
    rng = np.random.default_rng(7)
    for _ in range(300):
        nb = int(rng.integers(2, 34))
        hist = rng.integers(0, 6, size=nb).astype(np.uint64)
        if hist.sum() == 0:
            hist[0] = 1
        dists = np.repeat(np.arange(nb), hist.astype(np.int64))
        want = [float(x) for x in O.summary_numpy(dists.tolist()).values()]
        assert _lib.summary_from_hist(hist).tolist() == want


def test_summary_empty_raises_index_error(golden):
    with pytest.raises(IndexError) as ei:
        _lib.summary_from_hist(np.zeros(17, dtype=np.uint64))
    assert list(ei.value.args) == golden["errors"]["single"]["args"]


def test_limb_roundtrip():
    vals = [0, 1, 2 ** 63, 2 ** 64 - 1, 2 ** 64, 2 ** 100 + 12345, 3 ** 70]
    limbs = _lib.ints_to_limbs(vals)
    assert limbs.shape[1] == 2
    assert _lib.limbs_to_ints(limbs) == vals
    assert _lib.limbs_to_ints(_lib.ints_to_limbs([5, 7])) == [5, 7]


def test_tune_keys_match_header():
    """_lib.TUNE_KEYS names exactly the SCT_TUNE_* keys include/sctools_hip.h defines, with the
    same numbers, and every key round-trips through sct_tune_set / sct_tune_get (host only)."""
    import os
    import re
    hdr = open(os.path.join(os.path.dirname(__file__), "..", "include", "sctools_hip.h")).read()
    defined = {m.group(1).lower(): int(m.group(2)) for m in re.finditer(r"#define SCT_TUNE_(\w+)\s+(\d+)", hdr)}
    nkeys = defined.pop("nkeys")
    assert defined == _lib.TUNE_KEYS
    assert sorted(defined.values()) == list(range(1, nkeys))
    for name in _lib.TUNE_KEYS:
        with _lib.tuning(**{name: 7}):
            assert _lib.tune_get(name) == 7
        assert _lib.tune_get(name) == -1
