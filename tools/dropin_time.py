"""bench.py's paths.dropin_summary_737k alone (the drop-in summarize_hamming_distances call on
the 737,280-code set), with the C-level split of the histogram call.  One JSON line."""
import json
import sys
import time

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from sctools_amd import _lib, synthetic  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
n, L, seed = synthetic.CONFIGS[2]
codes = synthetic.whitelist_codes(n, L, seed)
hist = _lib.hamming_hist_allpairs(codes, 32)
out = {"dropin": bench.path_dropin(dev, 7, _lib.summary_from_hist(hist))}
# C-level: plan create / build / count / destroy on device-resident codes (the cached workspace)
d = torch.from_numpy(codes.view(np.int64)).cuda()
c = torch.zeros(53, dtype=torch.int64, device="cuda")
rows = []
for _ in range(5):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    p = _lib.AllPairsPlan(d.data_ptr(), n, 32)
    t1 = time.perf_counter()
    p.build()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    p.count(c.data_ptr())
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    p.close()
    t4 = time.perf_counter()
    rows.append([(t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3, (t4 - t3) * 1e3])
out["plan_ms"] = dict(zip(("create", "build_first", "count", "destroy"), np.median(np.array(rows), 0).tolist()))
t = time.perf_counter()
for _ in range(5):
    _lib.hamming_hist_allpairs(codes, 32)
out["hist_call_ms"] = (time.perf_counter() - t) / 5 * 1e3
t = time.perf_counter()
for _ in range(5):
    int(codes.max()).bit_length()
out["py_code_bits_ms"] = (time.perf_counter() - t) / 5 * 1e3
print(json.dumps(out))
