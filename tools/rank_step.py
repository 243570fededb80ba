"""Per-rank step time of the SPECTRAL path for N = 1, 2, 4, 8, emulated on one GPU (rank 0's
slice range; no process group, so no all-reduce and no inversion of the partial counts).
Shows the fixed per-step costs (build, launches, D2H) that strong scaling exposes."""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from sctools_amd import _lib, sharding, synthetic  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
n, L, seed = synthetic.CONFIGS[cfg]
codes = synthetic.whitelist_codes(n, L, seed)
d = torch.from_numpy(codes.view(np.int64)).cuda()
plan = _lib.AllPairsPlan(d.data_ptr(), n, 2 * L, scheme=_lib.SCHEME_SPECTRAL)
s = torch.cuda.current_stream()
sp = s.cuda_stream
counts = torch.zeros(plan.ncounts, dtype=torch.int64, device="cuda")
for world in (1, 2, 4, 8):
    b, e = sharding.item_range(plan.items, 0, world)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    bm, cm = [], []

    def step(rec):
        counts.zero_()
        if rec:
            evs[0].record(s)
        plan.build(sp, b, e)
        if rec:
            evs[1].record(s)
        plan.count(counts.data_ptr(), b, e, 0, sp)
        if rec:
            evs[2].record(s)
        h = counts.cpu()
        if rec:
            bm.append(evs[0].elapsed_time(evs[1]))
            cm.append(evs[1].elapsed_time(evs[2]))
        return h

    for _ in range(3):
        step(False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step(True)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps * 1e3
    print(json.dumps({"config": cfg, "world": world, "slices": e - b, "step_ms": dt,
                      "build_ms": float(np.median(bm)), "count_ms": float(np.median(cm)),
                      "ideal_ms_from_n1": None}), flush=True)
