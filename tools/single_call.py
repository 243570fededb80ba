"""Latency of one drop-in call, Barcodes.summarize_hamming_distances on the 737,280-code set
(host codes in, plan created, built, counted and destroyed inside the call), under SPECTRAL
chunk sizes; three calls each after one warm call.  One JSON line."""
import json
import sys
import time

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from sctools_amd import _lib, barcode, synthetic  # noqa: E402

n, L, seed = synthetic.CONFIGS[2]
codes = synthetic.whitelist_codes(n, L, seed)
b = barcode.Barcodes(dict.fromkeys((int(c) for c in codes), 1), L)
out = {}
for chunk in (262144, 65536, 262144):
    with _lib.tuning(spectral_chunk=chunk):
        b.summarize_hamming_distances()
        ts = []
        for _ in range(3):
            t = time.perf_counter()
            r = b.summarize_hamming_distances()
            ts.append((time.perf_counter() - t) * 1e3)
    out.setdefault(str(chunk), []).append(ts)
out["summary"] = {k: float(v) for k, v in r.items()}
print(json.dumps(out))
