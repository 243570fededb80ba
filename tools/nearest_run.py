"""Config 4 under a profiler: build the nearest-whitelist plan for the 737,280-code ThreeBit
whitelist and run 100M queries `--reps` times (tools/gpu_profile_r3.sh)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--scheme", type=int, default=0, help="SCT_TUNE_NEAREST_SCHEME (0 auto)")
    a = ap.parse_args()
    import numpy as np
    import torch
    from sctools_amd import _lib, synthetic
    n, L, seed = synthetic.CONFIGS[4]
    nq = synthetic.CONFIG4_QUERIES
    wl = synthetic.two_to_three(synthetic.whitelist_codes(n, L, seed), L)
    q, _, _ = synthetic.config4_queries(wl, nq, seed=4)
    d_wl = torch.from_numpy(wl.view(np.int64)).cuda()
    idx = torch.empty(nq, dtype=torch.int32, device="cuda")
    dist = torch.empty(nq, dtype=torch.uint8, device="cuda")
    with _lib.tuning(nearest_scheme=a.scheme):
        plan = _lib.NearestPlan(3, d_wl.data_ptr(), n, 3 * L, 1)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    plan.query(q.data_ptr(), nq, idx.data_ptr(), dist.data_ptr())
    e0.record()
    for _ in range(a.reps):
        plan.query(q.data_ptr(), nq, idx.data_ptr(), dist.data_ptr())
    e1.record()
    e1.synchronize()
    print("scheme", plan.info(), "ms per query pass", e0.elapsed_time(e1) / a.reps, flush=True)
    plan.close()


if __name__ == "__main__":
    main()
