"""Rank 0's share of config 2 at W ranks, emulated on one GPU (its slice range, no all-reduce), the
pipelined step bench.py times (ShardedAllPairs.run): ms per step for W = 1 and W, for a kernel trace.
  python tools/w8_share.py [W] [steps] [side|main]"""
import json
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from sctools_amd import _lib, sharding, synthetic  # noqa: E402

world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
build_on = sys.argv[3] if len(sys.argv) > 3 else "side"  # ShardedAllPairs.build_on
if len(sys.argv) > 4 and sys.argv[4] == "old":  # an A/B against a saved revision of the module
    from sctools_amd import _sharding_old as sharding  # noqa: F811
n, L, seed = synthetic.CONFIGS[2]
codes = synthetic.whitelist_codes(n, L, seed)
inv = _lib.counts_to_hist
out = {}
for w in (1, world):
    with sharding.ShardedAllPairs(codes, 2 * L) as job:
        job.begin, job.end = sharding.item_range(job.plan.items, 0, w)
        job.build_on = build_on
        _lib.counts_to_hist = inv if w == 1 else (lambda host, scheme, nbins: host)
        job.run(3)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        job.run(steps)
        torch.cuda.synchronize()
        out["w%d_ms" % w] = (time.perf_counter() - t0) / steps * 1e3
_lib.counts_to_hist = inv
out["linear_w%d_ms" % world] = out["w1_ms"] / world
out["build_on"] = build_on
print(json.dumps(out))
