"""Same-process A/B of the drop-in summary at 737K codes: Barcodes.summarize_hamming_distances()
as shipped (the C key loop also returns the keys' min / max) against the round-4 form of the same
call (numpy min for the sign check and numpy max for the code width after the conversion),
interleaved; results equal.  One JSON line."""
import json
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from sctools_amd import _lib, _pykeys, barcode, synthetic  # noqa: E402

n, L, seed = synthetic.CONFIGS[2]
codes = synthetic.whitelist_codes(n, L, seed)
b = barcode.Barcodes({int(c): 1 for c in codes}, L)


def old_form():
    arr = np.empty(len(b._data), dtype=np.int64)
    _pykeys.keys_to_int64(b._data, arr)
    arr = barcode.Barcodes._finish_int64(arr, True)  # numpy min
    hist = _lib.hamming_hist_allpairs(arr, distinct=True)  # numpy max
    return dict(zip(barcode._SUMMARY_KEYS, [np.float64(v) for v in _lib.summary_from_hist(hist)]))


ref = b.summarize_hamming_distances()
assert old_form() == ref
t = {"shipped": [], "round4_form": []}
for r in range(15):
    for k, f in (("shipped", b.summarize_hamming_distances), ("round4_form", old_form)):
        t0 = time.perf_counter()
        assert f() == ref
        t[k].append((time.perf_counter() - t0) * 1e3)
print(json.dumps({k: {"median_ms": float(np.median(v)), "all_ms": v} for k, v in t.items()}))
