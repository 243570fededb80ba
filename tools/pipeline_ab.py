"""Same-box A/B of ShardedAllPairs.step() in a loop against ShardedAllPairs.run() (steps
pipelined two deep), for rank 0's share at W = 1 and W = 8 (emulated on one GPU: the rank's
slice range, no all-reduce and no inversion of the partial counts).  Prints one JSON line per (W, mode, repeat)."""
import json
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from sctools_amd import _lib, sharding, synthetic  # noqa: E402

n, L, seed = synthetic.CONFIGS[2]
codes = synthetic.whitelist_codes(n, L, seed)
K = 20
with sharding.ShardedAllPairs(codes, 2 * L) as job:
    for world in (1, 8):
        job.begin, job.end = sharding.item_range(job.plan.items, 0, world)
        if world > 1:  # a rank's partial counts only invert after the all-reduce: skip it here
            _lib.counts_to_hist = lambda host, scheme, nbins: host
        for rep in range(3):
            for mode in ("step", "run"):
                if mode == "step":
                    for _ in range(3):
                        job.step()
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for _ in range(K):
                        job.step()
                    torch.cuda.synchronize()
                else:
                    job.run(3)
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    job.run(K)
                    torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) / K * 1e3
                print(json.dumps({"world": world, "mode": mode, "rep": rep, "ms_per_step": ms}), flush=True)
