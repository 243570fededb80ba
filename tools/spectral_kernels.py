"""Seed and tile kernel times of one SPECTRAL chunk (HIP events around back-to-back
launches, sct_allpairs_time_kernels), median over R calls; one JSON line (the kernels the
round-3 profile script traces for config 5).  Nothing is checked here."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from sctools_amd import _lib, synthetic  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
n, L, seed = synthetic.CONFIGS[cfg]
codes = synthetic.whitelist_codes(n, L, seed)
d = torch.from_numpy(codes.view(np.int64)).cuda()
p = _lib.AllPairsPlan(d.data_ptr(), n, 2 * L, scheme=_lib.SCHEME_SPECTRAL)
p.build()
s = torch.cuda.current_stream()
c = torch.zeros(p.ncounts, dtype=torch.int64, device="cuda")
c.zero_()
p.count(c.data_ptr(), 0, None, 0, s.cuda_stream)
torch.cuda.synchronize()
try:
    hist = p.counts_to_hist(c.cpu().numpy().view(np.uint64)).tolist()
except Exception as ex:  # ablation variants give counts that do not invert
    hist = "not invertible: %s" % type(ex).__name__
t = [p.time_kernels(c.data_ptr(), 0, None, 5, s.cuda_stream) for _ in range(rounds)]
print(json.dumps({"config": cfg, "env": {k: v for k, v in os.environ.items() if k.startswith("SCT_")},
                  "tile_ms": float(np.median([x["kernel_ms"] for x in t])),
                  "seed_ms": float(np.median([x["seed_ms"] for x in t])), "slices": t[0]["units"], "hist": hist}))
