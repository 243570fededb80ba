"""Summarise a tools/gpu_profile.sh run (gpurun_out/prof) into profiles/.

  python tools/summarize_profile.py --round r01 [--src gpurun_out/prof]

Writes profiles/<round>_kernel_stats.csv (rocprofv3 --kernel-trace --stats) and, for
the SPECTRAL tile kernel and the pair count kernel, profiles/pmc_{spectral,allpairs}_
<round>.json: per-launch PMC averages plus derived figures (clock from GRBM_GUI_ACTIVE / 8 XCDs / duration, VALU
lane-ops, HBM bytes from FETCH_SIZE/WRITE_SIZE in KiB with the gfx950 correction of
MI355X_MICROARCH.md §HBM: FETCH_SIZE counts half the bytes of wide streaming reads).
"""

import argparse
import collections
import csv
import glob
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def pmc_means(path, kernel_substr):
    agg = collections.defaultdict(float)
    cnt = collections.Counter()
    for f in glob.glob(os.path.join(path, "pmc*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if kernel_substr in r["Kernel_Name"]:
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
                cnt[r["Counter_Name"]] += 1
    return {k: agg[k] / cnt[k] for k in agg}


def last_calls_avg_ns(trace_csv, kernel_substr, k=5):
    """Mean duration of the kernel's last k dispatches in the trace: for bench.py these are
    the back-to-back launches of sct_allpairs_time_kernels, the same launches the bench
    line's kernel_ms times with HIP events."""
    if not os.path.exists(trace_csv):
        return None
    d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(trace_csv))
         if kernel_substr in r["Kernel_Name"]]
    return sum(d[-k:]) / len(d[-k:]) if d else None


def kernel_avg_ns(stats_csv, kernel_substr):
    for r in csv.DictReader(open(stats_csv)):
        if kernel_substr in r["Name"]:
            return float(r["AverageNs"]), int(r["Calls"])
    return None, 0


KERNELS = (("allpairs", "allpairs_count_kernel<8"), ("spectral", "tile_reg_p16_kernel"),
           ("spectral_seed", "seed_kernel<signed char"))


def summarize(src, dst, rnd, name, kernel, pairs):
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    avg_ns, calls = kernel_avg_ns(stats, kernel)
    if not calls:
        return None
    m = pmc_means(src, kernel)
    out = {"kernel": kernel, "trace_avg_ns": avg_ns, "trace_calls": calls, "pmc": m}
    if name.startswith("spectral"):
        out["trace_time_kernels_avg_ns"] = last_calls_avg_ns(os.path.join(src, "trace", "run_kernel_trace.csv"),
                                                             kernel)
        out["trace_note"] = ("trace_avg_ns averages every dispatch of the profiled bench run (warm-up and "
                             "timed steps included); trace_time_kernels_avg_ns the last 5, i.e. the "
                             "back-to-back launches the bench line's kernel_ms times with HIP events")
    if "GRBM_GUI_ACTIVE" in m and avg_ns:
        out["clock_ghz_estimate"] = m["GRBM_GUI_ACTIVE"] / 8 / avg_ns
    if "SQ_INSTS_VALU" in m:
        out["valu_wave_instructions"] = m["SQ_INSTS_VALU"]
        if name == "allpairs":
            out["valu_lane_ops_per_pair"] = m["SQ_INSTS_VALU"] * 64 / pairs
    if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
        fetch = m["FETCH_SIZE"] * 1024
        write = m["WRITE_SIZE"] * 1024
        out["hbm_bytes_per_launch_raw"] = fetch + write
        out["hbm_bytes_per_launch"] = 2 * fetch + write  # gfx950 FETCH_SIZE half-count correction
        out["note"] = ("FETCH_SIZE/WRITE_SIZE are KiB per dispatch; reads doubled per the gfx950 "
                       "correction (16-B-per-lane streaming reads).")
    for fn in ("pmc_%s_%s.json" % (name, rnd), "pmc_%s_latest.json" % name):
        with open(os.path.join(dst, fn), "w") as f:
            json.dump(dict(out, round=rnd), f, indent=1)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", default="r01")
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out", "prof"))
    ap.add_argument("--pairs", type=float, default=737280 * 737279 / 2)
    a = ap.parse_args()
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(a.src, "trace", "run_kernel_stats.csv"),
                os.path.join(dst, "%s_kernel_stats.csv" % a.round))
    for name, kernel in KERNELS:
        print(name, json.dumps(summarize(a.src, dst, a.round, name, kernel, a.pairs), indent=1))


if __name__ == "__main__":
    main()
