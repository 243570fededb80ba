"""WhitelistCorrector on config 4's 737,280-code ThreeBit whitelist from host arrays: its
construction (the device index) and ``nearest`` on one FASTQ flow piece's worth of queries
(3.7M, page-locked pool arrays as the encoder returns them, and pageable), each the median of 7
after 2 warm-ups.  One JSON line.  SCTOOLS_HIP_LIB selects the library (same-box A/B)."""
import json
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from sctools_amd import _lib, barcode, synthetic  # noqa: E402


def med(f, reps=9):
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        f()
        ts.append((time.perf_counter() - t) * 1e3)
    return float(np.median(ts[2:]))


n, L, seed = synthetic.CONFIGS[4]
wl = synthetic.two_to_three(synthetic.whitelist_codes(n, L, seed), L)
out = {"lib": _lib.lib()._name}
out["corrector_build_ms"] = med(lambda: barcode.WhitelistCorrector(wl, max_distance=1, encoding="ThreeBit").close())
c = barcode.WhitelistCorrector(wl, max_distance=1, encoding="ThreeBit")
rng = np.random.default_rng(5)
nq = 3_700_000
qp = _lib.pinned.empty(nq, np.uint64)
qp[:] = wl[rng.integers(0, wl.size, nq)]
qv = np.array(qp)  # pageable copy
ref = c.nearest(qv)
for name, q in (("query_pinned_ms", qp), ("query_pageable_ms", qv)):
    out[name] = med(lambda: c.nearest(q))
    idx, dist = c.nearest(q)
    assert np.array_equal(idx, ref[0]) and np.array_equal(dist, ref[1])
out["nq"] = nq
c.close()
print(json.dumps(out))
