"""A/B of config 4's nearest-whitelist query (100M ThreeBit queries vs the 737,280-code
whitelist, Hamming <= 1) under sct_tune knob sets, interleaved in one process: per variant a
plan made under its knobs, the query pass timed with HIP events (median over rounds of `reps`
passes), and the outputs checked identical to the first variant's.  One JSON line.
Usage: ab_nearest_tune.py ROUNDS 'nearest_scheme=0' 'nearest_scheme=1' ..."""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from sctools_amd import _lib, synthetic  # noqa: E402

rounds = int(sys.argv[1])
variants = [dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in a.split(",") if kv) for a in sys.argv[2:]]
n, L, seed = synthetic.CONFIGS[4]
nq = synthetic.CONFIG4_QUERIES
wl = synthetic.two_to_three(synthetic.whitelist_codes(n, L, seed), L)
q, _, _ = synthetic.config4_queries(wl, nq, seed=4)
d_wl = torch.from_numpy(wl.view(np.int64)).cuda()
plans = []
for v in variants:
    with _lib.tuning(**v):
        plans.append(_lib.NearestPlan(3, d_wl.data_ptr(), n, 3 * L, 1))
idx = [torch.empty(nq, dtype=torch.int32, device="cuda") for _ in variants]
dist = [torch.empty(nq, dtype=torch.uint8, device="cuda") for _ in variants]
times = [[] for _ in variants]
reps = 5
for r in range(rounds):
    for i, v in enumerate(variants):
        with _lib.tuning(**v):
            plans[i].query(q.data_ptr(), nq, idx[i].data_ptr(), dist[i].data_ptr())
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(reps):
                plans[i].query(q.data_ptr(), nq, idx[i].data_ptr(), dist[i].data_ptr())
            b.record()
            b.synchronize()
            times[i].append(a.elapsed_time(b) / reps)
out = {"config": 4, "queries": nq, "rounds": rounds, "time": time.strftime("%Y-%m-%d %H:%M:%S"), "variants": []}
for i, v in enumerate(variants):
    same = bool(torch.equal(idx[i], idx[0]) and torch.equal(dist[i], dist[0]))
    out["variants"].append({"tune": v, "info": plans[i].info(), "ms": float(np.median(times[i])), "all_ms": times[i],
                            "outputs_equal_first": same})
print(json.dumps(out))
