"""Where the one-shot drop-in call goes (737K set): the mapping -> numpy conversion
(Barcodes.codes_array), the histogram call (H2D, plan, build, count, destroy), the summary,
and a bare plan create / destroy.  One JSON line."""
import sys, time, json
sys.path.insert(0, ".")
import numpy as np, torch
from sctools_amd import _lib, barcode, synthetic
n, L, seed = synthetic.CONFIGS[2]
codes = synthetic.whitelist_codes(n, L, seed)
b = barcode.Barcodes(dict.fromkeys((int(c) for c in codes), 1), L)
b.summarize_hamming_distances()
out = {}
for it in range(3):
    t0 = time.perf_counter(); arr = b.codes_array(); t1 = time.perf_counter()
    h = _lib.hamming_hist_allpairs(arr); t2 = time.perf_counter()
    s = _lib.summary_from_hist(h); t3 = time.perf_counter()
    out.setdefault("codes_array_ms", []).append((t1 - t0) * 1e3)
    out.setdefault("hist_ms", []).append((t2 - t1) * 1e3)
    out.setdefault("summary_ms", []).append((t3 - t2) * 1e3)
d = torch.from_numpy(codes.view(np.int64)).cuda(); torch.cuda.synchronize()
for it in range(3):
    t0 = time.perf_counter(); p = _lib.AllPairsPlan(d.data_ptr(), n, 32); torch.cuda.synchronize(); t1 = time.perf_counter()
    p.close(); torch.cuda.synchronize(); t2 = time.perf_counter()
    out.setdefault("plan_create_ms", []).append((t1 - t0) * 1e3)
    out.setdefault("plan_destroy_ms", []).append((t2 - t1) * 1e3)
print(json.dumps(out))
