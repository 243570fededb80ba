"""Multi-limb all-pairs kernel (sct_allpairs_wide) throughput: n random ThreeBit 28-bp
codes (84 bits = 2 limbs), device-resident, HIP-event time of the count over all items;
one JSON line.  argv: n [repeats]."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from sctools_amd import _lib  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rng = np.random.default_rng(7)
L = 28
lo = np.zeros(n, dtype=np.uint64)
hi = np.zeros(n, dtype=np.uint64)
for p in range(L):  # ThreeBit A C G T = 2 1 3 4 at 3 bits per base, MSB-first
    v = np.array([2, 1, 3, 4], dtype=np.uint64)[rng.integers(0, 4, n)]
    sh = 3 * (L - 1 - p)
    if sh >= 64:
        hi |= v << np.uint64(sh - 64)
    elif sh + 3 > 64:
        lo |= v << np.uint64(sh)
        hi |= v >> np.uint64(64 - sh)
    else:
        lo |= v << np.uint64(sh)
limbs = np.stack([lo, hi], axis=1)
items, nbins = _lib.wide_geometry(n, 2)
d = torch.from_numpy(limbs.view(np.int64)).cuda()
h = torch.zeros(nbins, dtype=torch.int64, device="cuda")
s = torch.cuda.current_stream()
lib = _lib.lib()
_lib.check(lib.sct_allpairs_wide(d.data_ptr(), n, 2, 0, items, h.data_ptr(), nbins, s.cuda_stream))
torch.cuda.synchronize()
ts = []
for _ in range(reps):
    h.zero_()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    _lib.check(lib.sct_allpairs_wide(d.data_ptr(), n, 2, 0, items, h.data_ptr(), nbins, s.cuda_stream))
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
pairs = n * (n - 1) // 2
hist = h.cpu().numpy().view(np.uint64)
assert int(hist.sum()) == pairs
ms = float(np.median(ts))
print(json.dumps({"n": n, "words": 2, "pairs": pairs, "median_ms": ms, "pairs_per_s": pairs / (ms * 1e-3),
                  "hist_head": hist[:20].tolist()}))
