"""Where AUTO should switch from the pair-enumerating MOMENTS kernel to SPECTRAL: the whole
pipelined step (ShardedAllPairs.run: build, count, read-back, inversion) of both schemes on
seeded random 16-bp sets of the given sizes, interleaved, medians over rounds.  One JSON line
per size; the histograms of the two schemes must agree.

  python tools/crossover.py 250000 300000 350000 400000 450000 500000
"""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from sctools_amd import _lib, sharding, synthetic  # noqa: E402

ROUNDS, STEPS = 5, 4


def step_ms(job):
    job.run(1)
    torch.cuda.synchronize()
    t = time.perf_counter()
    hists = job.run(STEPS)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / STEPS * 1e3, hists[-1]


for n in [int(x) for x in sys.argv[1:]]:
    codes = synthetic.whitelist_codes(n, 16, seed=n)
    jobs = {name: sharding.ShardedAllPairs(codes, 32, scheme=sch)
            for name, sch in (("moments", _lib.SCHEME_MOMENTS), ("spectral", _lib.SCHEME_SPECTRAL))}
    ms = {k: [] for k in jobs}
    hist = {}
    for _ in range(ROUNDS):
        for k, job in jobs.items():
            t, h = step_ms(job)
            ms[k].append(t)
            hist[k] = h
    for job in jobs.values():
        job.close()
    print(json.dumps({"n": n, "moments_ms": float(np.median(ms["moments"])),
                      "spectral_ms": float(np.median(ms["spectral"])),
                      "same_hist": bool(np.array_equal(hist["moments"], hist["spectral"]))}), flush=True)
