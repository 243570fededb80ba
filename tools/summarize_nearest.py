"""Summarise tools/gpu_prof_nearest.sh (gpurun_out/profn_{after,before}) into
profiles/pmc_nearest_<round>_<variant>.json: per-launch PMC of nearest_query_kernel, per
query (L2 hits / misses / Infinity-Cache-or-DRAM read requests), the trace's average
duration and the bench line's HIP-event median."""

import argparse
import json
import os
import shutil
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from summarize_profile import kernel_avg_ns, pmc_means  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", default="r02")
    ap.add_argument("--queries", type=float, default=1e8)
    a = ap.parse_args()
    for variant in ("after", "csr", "before"):
        src = os.path.join(ROOT, "gpurun_out", "profn_" + variant)
        stats = os.path.join(src, "trace", "run_kernel_stats.csv")
        if not os.path.exists(stats):
            continue
        k = "oa_query_kernel" if variant == "after" else "nearest_query_kernel"
        avg_ns, calls = kernel_avg_ns(stats, k)
        m = pmc_means(src, k)
        per_q = {c: v / a.queries for c, v in m.items() if c.startswith(("TCC", "TCP", "SQ_INSTS"))}
        bench = None
        try:
            for line in open(os.path.join(src, "bench.json")):
                bench = json.loads(line)
        except (OSError, ValueError):
            pass
        out = {"kernel": k, "variant": variant, "queries_per_launch": a.queries, "trace_avg_ns": avg_ns,
               "trace_calls": calls, "pmc_per_launch": m, "per_query": per_q, "bench": bench}
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            out["hbm_bytes_per_launch"] = 2 * m["FETCH_SIZE"] * 1024 + m["WRITE_SIZE"] * 1024
        if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m:
            out["l2_hit_rate"] = m["TCC_HIT_sum"] / max(1.0, m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
        dst = os.path.join(ROOT, "profiles", "pmc_nearest_%s_%s.json" % (a.round, variant))
        with open(dst, "w") as f:
            json.dump(out, f, indent=1)
        shutil.copy(stats, os.path.join(ROOT, "profiles", "%s_nearest_%s_kernel_stats.csv" % (a.round, variant)))
        print(dst, json.dumps({"trace_ms": avg_ns / 1e6 if avg_ns else None, "per_query": per_q,
                               "l2_hit_rate": out.get("l2_hit_rate")}))


if __name__ == "__main__":
    main()
