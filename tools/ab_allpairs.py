"""Interleaved A/B timing of all-pairs count-kernel variants in ONE process.

(Round 2 tool.  SCT_ALLPAIRS_VARIANT is read only by the ablation build (make ablation); grid,
grab and the SPECTRAL chunk are sct_tune_set keys since round 3 -- tools/ab_seed_tune.py and
tools/ab_nearest_tune.py are the current A/B drivers.)
Variants are selected at plan creation through SCT_ALLPAIRS_VARIANT / _GRID / _GRAB and
the count scheme (s=0 SUBSETS, s=1 MOMENTS, s=2 SPECTRAL with chunk=slices per pass); each round times every variant once (HIP
events on the launch stream: the count kernel, and the moments pass separately); prints
the median and min per variant and checks that all variants give identical histograms.

  python tools/ab_allpairs.py --config 2 --rounds 7 --variants "v=2,s=0" "v=3,s=1" "v=1,grid=2048"
"""

import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from sctools_amd import _lib, synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--variants", nargs="+", default=["v=2", "v=1"])
    a = ap.parse_args()
    n, L, seed = synthetic.CONFIGS[a.config]
    codes = synthetic.whitelist_codes(n, L, seed)
    d = torch.from_numpy(codes.view(np.int64)).cuda()
    plans = []
    for v in a.variants:
        kv = dict(x.split("=") for x in v.split(","))
        os.environ["SCT_ALLPAIRS_VARIANT"] = kv.get("v", "2")
        for key, env in (("grid", "SCT_ALLPAIRS_GRID"), ("grab", "SCT_ALLPAIRS_GRAB"),
                         ("chunk", "SCT_SPECTRAL_CHUNK")):
            if key in kv:
                os.environ[env] = kv[key]
            else:
                os.environ.pop(env, None)
        p = _lib.AllPairsPlan(d.data_ptr(), n, 2 * L, scheme=int(kv.get("s", "-1")))
        p.build()
        plans.append((v, p))
    s = torch.cuda.current_stream()
    times = {v: [] for v, _ in plans}
    mtimes = {v: [] for v, _ in plans}
    btimes = {v: [] for v, _ in plans}
    ref = None
    for _ in range(a.rounds):
        for v, p in plans:
            c = torch.zeros(p.ncounts, dtype=torch.int64, device="cuda")
            eb, em, e0, e1 = (torch.cuda.Event(enable_timing=True) for _ in range(4))
            eb.record(s)
            p.build(s.cuda_stream)
            em.record(s)
            p.moments(c.data_ptr(), stream=s.cuda_stream)
            e0.record(s)
            p.count(c.data_ptr(), stream=s.cuda_stream)
            e1.record(s)
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1))
            mtimes[v].append(em.elapsed_time(e0))
            btimes[v].append(eb.elapsed_time(em))
            if int(dict(x.split("=") for x in v.split(",")).get("v", "2")) >= 10:
                continue  # ablation builds compute wrong counts by design
            h = p.counts_to_hist(c.cpu().numpy().view(np.uint64))
            if ref is None:
                ref = h
            assert np.array_equal(ref, h), v
    pairs = plans[0][1].pairs
    out = {v: {"median_ms": float(np.median(t)), "min_ms": float(np.min(t)),
               "moments_ms": float(np.median(mtimes[v])), "build_ms": float(np.median(btimes[v])),
               "scheme": dict(plans)[v].scheme,
               "pairs_per_s": pairs / (np.median(t) * 1e-3)} for v, t in times.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
