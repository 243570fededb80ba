"""Same-box A/B of the SPECTRAL kernels across library builds: config 2's seed and tile kernels
timed apart (sct_allpairs_time_kernels: back-to-back launches over all 2^18 slices bracketed by
HIP events), each library in its own process, rounds interleaved.

  python tools/tile_ab.py base= sqabl=sctools_amd/libsctools_hip_sqabl.so [--rounds 3] [--config 2]"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import json, sys
import numpy as np, torch
sys.path.insert(0, %r)
from sctools_amd import _lib, synthetic
n, L, seed = synthetic.CONFIGS[%d]
codes = synthetic.whitelist_codes(n, L, seed)
d = torch.from_numpy(codes.view(np.int64)).cuda()
p = _lib.AllPairsPlan(d.data_ptr(), n, 2 * L, scheme=_lib.SCHEME_SPECTRAL)
p.build()
c = torch.zeros(p.ncounts, dtype=torch.int64, device="cuda")
r = p.time_kernels(c.data_ptr(), 0, p.items, repeats=10)
print(json.dumps(r))
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--config", type=int, default=2)
    a = ap.parse_args()
    res = {}
    for rnd in range(a.rounds):
        for v in a.variants:
            name, lib = v.split("=", 1)
            env = dict(os.environ)
            if lib:
                env["SCTOOLS_HIP_LIB"] = os.path.join(ROOT, lib)
            out = subprocess.run([sys.executable, "-c", CHILD % (ROOT, a.config)], env=env, capture_output=True,
                                 text=True, timeout=300)
            if out.returncode != 0:
                print(json.dumps({"variant": name, "error": out.stderr[-800:]}), flush=True)
                return 3
            r = json.loads(out.stdout.strip().splitlines()[-1])
            r.update(variant=name, round=rnd)
            print(json.dumps(r), flush=True)
            res.setdefault(name, []).append(r)
    summ = {k: {"tile_ms_min": min(x["kernel_ms"] for x in v), "seed_ms_min": min(x["seed_ms"] for x in v)}
            for k, v in res.items()}
    print(json.dumps({"summary": summ}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
