"""Same-box A/B of how ShardedAllPairs.run()'s count waits for the side-stream build
(``build_wait`` "gpu": a cross-queue wait of the main stream on the build's event, "host": the host
waits for that event before enqueuing the count) at W = 1 and for rank 0's share at W = 8
(emulated on one GPU: the rank's slice range, no all-reduce).  One JSON line per (W, mode, repeat)."""
import json
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from sctools_amd import _lib, sharding, synthetic  # noqa: E402

n, L, seed = synthetic.CONFIGS[2]
codes = synthetic.whitelist_codes(n, L, seed)
K = 20
inv = _lib.counts_to_hist
for world in (1, 8):
    for rep in range(3):
        for mode in ("gpu", "host"):
            with sharding.ShardedAllPairs(codes, 2 * L) as job:
                job.build_wait = mode
                job.begin, job.end = sharding.item_range(job.plan.items, 0, world)
                _lib.counts_to_hist = inv if world == 1 else (lambda host, scheme, nbins: host)
                job.run(3)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                hists = job.run(K)
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) / K * 1e3
                same = all((h == hists[0]).all() for h in hists)
            print(json.dumps({"world": world, "mode": mode, "rep": rep, "ms_per_step": ms, "steps_agree": bool(same)}),
                  flush=True)
_lib.counts_to_hist = inv
