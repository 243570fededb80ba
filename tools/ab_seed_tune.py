"""A/B of SPECTRAL kernel variants selected through sct_tune_set, interleaved in one process:
for each variant (a dict of tune keys) the whole count's histogram (checked equal to the
first variant's and, when --oracle, to the C oracle) and the seed / tile kernel times of
one chunk (time_kernels, HIP events around back-to-back launches) and the build + count of
the whole job (count_ms), medians over rounds; one plan per variant, made under its knobs.
Usage: ab_seed_tune.py CONFIG ROUNDS 'spectral_chunk=65536' 'spectral_chunk=32768' ...
(round 3 used it with two A/B-only keys, spectral_seed / spectral_seed_walks, since removed)
Prints one JSON line."""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from sctools_amd import _lib, synthetic  # noqa: E402

cfg, rounds = int(sys.argv[1]), int(sys.argv[2])
variants = [dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in a.split(",") if kv) for a in sys.argv[3:]]
n, L, seed = synthetic.CONFIGS[cfg]
codes = synthetic.whitelist_codes(n, L, seed)
d = torch.from_numpy(codes.view(np.int64)).cuda()
s = torch.cuda.current_stream()
sp = s.cuda_stream
plans = []  # one plan per variant, created under its knobs (some decide the plan's layout)
for v in variants:
    with _lib.tuning(**v):
        p = _lib.AllPairsPlan(d.data_ptr(), n, 2 * L, scheme=_lib.SCHEME_SPECTRAL)
        p.build(sp, 0, p.items)
    plans.append(p)
c = torch.zeros(plans[0].ncounts, dtype=torch.int64, device="cuda")


def run_variant(v, plan):
    with _lib.tuning(**v):
        plan.build(sp, 0, plan.items)
        c.zero_()
        plan.count(c.data_ptr(), 0, None, 0, sp)
        torch.cuda.synchronize()
        hist = plan.counts_to_hist(c.cpu().numpy().view(np.uint64)).tolist()
        t = plan.time_kernels(c.data_ptr(), 0, None, 5, sp)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        c.zero_()
        a.record(s)
        plan.build(sp, 0, plan.items)
        plan.count(c.data_ptr(), 0, None, 0, sp)
        b.record(s)
        torch.cuda.synchronize()
        return hist, t["seed_ms"], t["kernel_ms"], a.elapsed_time(b)


res = [{"seed": [], "tile": [], "count": [], "hist": None} for _ in variants]
for r in range(rounds):
    for i, v in enumerate(variants):
        h, sm, tm, cm = run_variant(v, plans[i])
        res[i]["seed"].append(sm)
        res[i]["tile"].append(tm)
        res[i]["count"].append(cm)
        if res[i]["hist"] is None:
            res[i]["hist"] = h
        elif res[i]["hist"] != h:
            res[i]["hist_unstable"] = True
ref = res[0]["hist"]
out = {"config": cfg, "n": n, "rounds": rounds, "time": time.strftime("%Y-%m-%d %H:%M:%S"), "variants": []}
for v, r in zip(variants, res):
    out["variants"].append({"tune": v, "info": plans[variants.index(v)].spectral_info(), "seed_ms": float(np.median(r["seed"])), "tile_ms": float(np.median(r["tile"])),
                            "count_ms": float(np.median(r["count"])), "seed_all": r["seed"],
                            "hist_equal_first": r["hist"] == ref, "unstable": r.get("hist_unstable", False)})
out["hist"] = ref
print(json.dumps(out))
