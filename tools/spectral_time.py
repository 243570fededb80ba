"""Time one SPECTRAL count (seed + tile passes) on a config, HIP events, median of R runs.
Round 2 used it with the ablation library and SCT_SPECTRAL_ABL=1..4 (SPECTRAL ablations since
removed from the sources; the ablation build now only varies the pair kernel).  Nothing is
checked here."""
import json
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
t = []
for _ in range(rounds + 1):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    p.count(c.data_ptr(), stream=s.cuda_stream)
    e1.record(s)
    torch.cuda.synchronize()
    t.append(e0.elapsed_time(e1))
print(json.dumps({"config": cfg, "median_ms": float(np.median(t[1:])), "min_ms": float(np.min(t[1:]))}))
