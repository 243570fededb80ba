"""Where the SPECTRAL step's time goes beyond the kernels' isolated times: the seed and tile
kernels timed apart (back-to-back launches of one kernel, `time_kernels`), against one
65,536-slice chunk counted as seed + tile pairs (the step's alternation), against the whole
262,144-slice count, all on the bench's 737K set.  Prints one JSON line."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from sctools_amd import _lib, synthetic  # noqa: E402

n, L, seed = synthetic.CONFIGS[2]
codes = synthetic.whitelist_codes(n, L, seed)
d = torch.from_numpy(codes.view(np.int64)).cuda()
plan = _lib.AllPairsPlan(d.data_ptr(), n, 2 * L, scheme=_lib.SCHEME_SPECTRAL)
s = torch.cuda.current_stream()
sp = s.cuda_stream
counts = torch.zeros(plan.ncounts, dtype=torch.int64, device="cuda")
plan.build(sp, 0, plan.items)
out = {}


def timed(fn, reps):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    a.record(s)
    for _ in range(reps):
        fn()
    b.record(s)
    b.synchronize()
    return a.elapsed_time(b) / reps


for rep in range(3):
    tk = plan.time_kernels(counts.data_ptr(), 0, plan.items, 5, sp)
    out.setdefault("isolated_seed_ms", []).append(tk["seed_ms"])
    out.setdefault("isolated_tile_ms", []).append(tk["kernel_ms"])
    out.setdefault("chunk_pair_ms", []).append(timed(lambda: plan.count(counts.data_ptr(), 0, 65536, 0, sp), 5))
    out.setdefault("full_count_ms", []).append(timed(lambda: plan.count(counts.data_ptr(), 0, plan.items, 0, sp), 5))
    out.setdefault("build_plus_count_ms", []).append(
        timed(lambda: (plan.build(sp, 0, plan.items), plan.count(counts.data_ptr(), 0, plan.items, 0, sp)), 5))
print(json.dumps(out))
