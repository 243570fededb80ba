"""Interleaved A/B timing of all-pairs count-kernel variants in ONE process.

Variants are selected at plan creation through SCT_ALLPAIRS_UNROLL / SCT_ALLPAIRS_GRID;
each round times every variant once (HIP events on the launch stream); prints the
median and min per variant and checks that all variants produce identical counts.

  python tools/ab_allpairs.py --config 2 --rounds 7 --variants "v=2" "v=1" "v=1,grid=2048"
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
        for key in ("grid", "grab"):
            env = "SCT_ALLPAIRS_" + key.upper()
            if key in kv:
                os.environ[env] = kv[key]
            else:
                os.environ.pop(env, None)
        p = _lib.AllPairsPlan(d.data_ptr(), n, 2 * L)
        p.build()
        plans.append((v, p))
    s = torch.cuda.current_stream()
    times = {v: [] for v, _ in plans}
    ref = None
    for _ in range(a.rounds):
        for v, p in plans:
            c = torch.zeros(p.nbins, dtype=torch.int64, device="cuda")
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            p.count(c.data_ptr(), stream=s.cuda_stream)
            e1.record(s)
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1))
            cc = c.cpu().numpy()
            if int(dict(x.split("=") for x in v.split(",")).get("v", "2")) >= 10:
                continue  # ablation builds compute wrong counts by design
            if ref is None:
                ref = cc
            assert np.array_equal(ref, cc), v
    pairs = plans[0][1].pairs
    out = {v: {"median_ms": float(np.median(t)), "min_ms": float(np.min(t)),
               "pairs_per_s": pairs / (np.median(t) * 1e-3)} for v, t in times.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
