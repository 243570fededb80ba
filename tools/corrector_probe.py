"""WhitelistCorrector construction (the device index of config 4's 737,280-code ThreeBit
whitelist from a host array) timed alone, median of 7 after 2 warm-ups.  One JSON line."""
import json
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from sctools_amd import barcode, synthetic  # noqa: E402

n, L, seed = synthetic.CONFIGS[4]
wl = synthetic.two_to_three(synthetic.whitelist_codes(n, L, seed), L)
ts = []
for _ in range(9):
    t = time.perf_counter()
    c = barcode.WhitelistCorrector(wl, max_distance=1, encoding="ThreeBit")
    ts.append((time.perf_counter() - t) * 1e3)
    c.close()
print(json.dumps({"corrector_build_ms": float(np.median(ts[2:])), "all_ms": ts}))
