"""What the per-step plan build costs ShardedAllPairs.run() (diagnostic, not a bench path): steps
timed with the build as shipped and with each plan's build skipped after its first (the tables
are those of the same codes, so every histogram stays the same), at W = 1 and for rank 0's share
at W = 8 (emulated on one GPU: the rank's slice range, no all-reduce).  One JSON line per
(W, mode, repeat)."""
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
        for mode in ("build", "nobuild"):
            with sharding.ShardedAllPairs(codes, 2 * L) as job:
                job.begin, job.end = sharding.item_range(job.plan.items, 0, world)
                _lib.counts_to_hist = inv if world == 1 else (lambda host, scheme, nbins: host)
                job.run(3)
                torch.cuda.synchronize()
                if mode == "nobuild":
                    for p in job._pipe["plans"]:
                        p.build = lambda *a, **k: None
                t0 = time.perf_counter()
                hists = job.run(K)
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) / K * 1e3
                same = all((h == hists[0]).all() for h in hists)
            print(json.dumps({"world": world, "mode": mode, "rep": rep, "ms_per_step": ms, "steps_agree": bool(same)}),
                  flush=True)
_lib.counts_to_hist = inv
