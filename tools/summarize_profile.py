"""Summarise a tools/gpu_profile_r3.sh run into profiles/.

  python tools/summarize_profile.py --round r03 [--src gpurun_out/prof3]

Writes profiles/<round>_kernel_stats.csv (rocprofv3 --kernel-trace --stats of the exact
default bench command), profiles/<round>_nearest_kernel_stats.csv (config 4's queries), and
per kernel profiles/pmc_<name>_<round>.json: the trace average, per-launch PMC averages and
derived figures -- clock = GRBM_GUI_ACTIVE / 8 XCDs / duration; VALU / matrix-pipe busy
fractions of the SIMD cycles (SQ_ACTIVE_INST_VALU counts quad-cycles); HBM bytes from
FETCH_SIZE / WRITE_SIZE (KiB) with the gfx950 correction of MI355X_MICROARCH.md §HBM
(FETCH_SIZE counts half the bytes of wide streaming reads); L2 hit rate and memory-side read
requests (TCC_EA0_RDREQ) per launch.
"""

import argparse
import collections
import csv
import glob
import json
import os
import statistics
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIMDS = 1024

# (name, kernel-name substring, pmc pass dirs prefix, trace dir, units per launch, unit)
KERNELS = (
    ("spectral_seed", "seed_sm_kernel", "pmc", "trace", 262144, "slices"),
    ("spectral", "tile_reg_kernel", "pmc", "trace", 262144, "slices"),
    ("spectral_seed_int16", "seed_kernel<short>", "pmc", "trace", 65536, "slices"),
    ("spectral_seed16", "seed16_sm_kernel", "s5pmc", "s5trace", 65536, "slices of 2^16"),
    ("spectral16", "tile16_kernel", "s5pmc", "s5trace", 65536, "slices of 2^16"),
    ("nearest", "halves_query_kernel<3, true>", "npmc", "ntrace", 100_000_000, "queries"),
    ("nearest_index", "halves_index_kernel", "npmc", "ntrace", 100_000_000, "queries"),
    ("whitelist_spec16", "whitelist_spec16_kernel", "ipmc", "itrace", 3_686_400, "lines"),
    ("whitelist_fused", "whitelist_fused_kernel", "ipmc", "itrace", 3_686_400, "lines"),
    ("fastq_range", "fastq_range_kernel", "ipmc", "itrace", 20_000_000, "records"),
    ("whitelist_count", "wl_count_kernel", "ipmc", "itrace", 3_686_400, "lines"),
    ("fastq_count", "fq_count_kernel", "ipmc", "itrace", 20_000_000, "records"),
    ("base_frequency16", "base_frequency16_kernel", "ipmc", "itrace", 3_686_400, "codes"),
    ("base_frequency_reduce", "base_frequency_reduce_kernel", "ipmc", "itrace", 3_686_400, "codes"),
)


def timed_window(src, trace, kernel_substr, last, skip=5):
    """Mean duration of the bench's timed dispatches of a kernel in a kernel trace: in start
    order, the headline job's `skip` warm-up dispatches come first and its `last` timed ones
    next (the side paths -- the drop-in summary too -- run after the headline and are not
    counted), i.e. the launches the bench line's HIP events time."""
    path = os.path.join(src, trace, "run_kernel_trace.csv")
    if not os.path.exists(path):
        return None
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(path))
                  if kernel_substr in r["Kernel_Name"])
    d = [e - b for b, e in rows]
    if not d:
        return None
    w = d[skip:skip + last] or d[-last:]
    return {"kernel": kernel_substr, "dispatches": len(d), "window": len(w), "window_first": skip,
            "avg_ns": sum(w) / len(w), "all_avg_ns": sum(d) / len(d)}


def pmc_means(src, prefix, kernel_substr):
    """Per counter, the median over the profiled dispatches of the kernel: a plan's first
    dispatch into its freshly allocated 4 GiB intermediate runs up to 10x the cycles of the
    others under the counter passes, and a mean over a handful of dispatches follows it."""
    vals = collections.defaultdict(list)
    for f in glob.glob(os.path.join(src, prefix + "[0-9]*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if kernel_substr in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: statistics.median(v) for k, v in vals.items()}


def kernel_avg_ns(stats_csv, kernel_substr):
    if not os.path.exists(stats_csv):
        return None, 0
    for r in csv.DictReader(open(stats_csv)):
        if kernel_substr in r["Name"]:
            return float(r["AverageNs"]), int(r["Calls"])
    return None, 0


def summarize(src, dst, rnd, name, kernel, prefix, trace, units, unit, window=None):
    avg_ns, calls = kernel_avg_ns(os.path.join(src, trace, "run_kernel_stats.csv"), kernel)
    if window:  # the headline's full-size timed dispatches (the side paths launch smaller ones)
        avg_ns, calls = window["avg_ns"], window["window"]
    m = pmc_means(src, prefix, kernel)
    if not calls and not m:
        return None
    out = {"kernel": kernel, "trace_avg_ns": avg_ns, "trace_calls": calls, "units_per_launch": units, "unit": unit,
           "pmc": m}
    if "GRBM_GUI_ACTIVE" in m and avg_ns:
        cycles = m["GRBM_GUI_ACTIVE"] / 8
        out["clock_ghz_estimate"] = cycles / avg_ns
        if "SQ_ACTIVE_INST_VALU" in m:
            out["valu_busy_frac"] = 4 * m["SQ_ACTIVE_INST_VALU"] / (SIMDS * cycles)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            out["mfma_busy_frac"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * cycles)
    if "SQ_WAVE_CYCLES" in m:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if k in m:
                out[k.lower()[3:] + "_frac_of_wave_cycles"] = m[k] / m["SQ_WAVE_CYCLES"]
    if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
        fetch, write = m["FETCH_SIZE"] * 1024, m["WRITE_SIZE"] * 1024
        out["hbm_bytes_per_launch_raw"] = fetch + write
        out["hbm_bytes_per_launch"] = 2 * fetch + write  # gfx950 FETCH_SIZE half-count correction
        out["hbm_bytes_per_unit"] = out["hbm_bytes_per_launch"] / units
    if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m and m["TCC_HIT_sum"] + m["TCC_MISS_sum"] > 0:
        out["l2_hit_rate"] = m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
        out["l2_requests_per_unit"] = (m["TCC_HIT_sum"] + m["TCC_MISS_sum"]) / units
    if "TCC_EA0_RDREQ_sum" in m:
        out["ea_read_requests_per_unit"] = m["TCC_EA0_RDREQ_sum"] / units
    out["note"] = ("per-launch medians over the profiled dispatches of the kernel; FETCH_SIZE/WRITE_SIZE are KiB "
                   "per dispatch, reads doubled per the gfx950 correction; busy fractions are of 1024 SIMDs x "
                   "the profiled run's cycles")
    with open(os.path.join(dst, "pmc_%s_%s.json" % (name, rnd)), "w") as f:
        json.dump(dict(out, round=rnd), f, indent=1)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", default="r03")
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out", "prof3"))
    a = ap.parse_args()
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    for trace, fn in (("trace", "%s_kernel_stats.csv"), ("ntrace", "%s_nearest_kernel_stats.csv"),
                      ("s5trace", "%s_config5_kernel_stats.csv"), ("itrace", "%s_ingest_kernel_stats.csv")):
        src = os.path.join(a.src, trace, "run_kernel_stats.csv")
        if os.path.exists(src):
            shutil.copy(src, os.path.join(dst, fn % a.round))
    ap_steps = int(os.environ.get("BENCH_STEPS", "20"))
    # the headline's untimed dispatches: bench.py's settle steps (30 at N = 1) + its warmup
    ap_warm = int(os.environ.get("BENCH_WARMUP", "5")) + int(os.environ.get("BENCH_SETTLE", "30"))
    win = {k: timed_window(a.src, "trace", k, ap_steps, ap_warm) for k in ("tile_reg_kernel", "seed_sm_kernel")}
    # the profiled command's own bench line: its live HIP-event kernel times, same box and run
    live = {}
    log = os.path.join(a.src, "trace.log")
    if os.path.exists(log):
        for line in open(log):
            if line.startswith("{") and '"roofline"' in line:
                r = json.loads(line)["roofline"]
                live = {"tile_reg_kernel": r.get("kernel_ms"), "seed_sm_kernel": (r.get("other_kernel") or {}).get("ms")}
    for k, w in win.items():
        if w and live.get(k):
            w["live_ms_same_run"] = live[k]
            w["live_vs_trace_same_run"] = live[k] / (w["avg_ns"] * 1e-6) - 1.0
    with open(os.path.join(dst, "%s_timed_dispatches.json" % a.round), "w") as f:
        json.dump({"command": "python3 bench.py --gpus 1 --steps %d --warmup %d" % (ap_steps, ap_warm), "kernels": win,
                   "note": "rocprofv3 kernel trace of the command; avg_ns = the kernel's dispatches "
                           "[window_first, window_first + window) in start order (the headline's timed steps, "
                           "after its warm-up), all_avg_ns = every dispatch; live_ms_same_run = "
                           "the HIP-event kernel time the same profiled command printed (same box, same run)"},
                  f, indent=1)
    print("timed window", json.dumps(win))
    for name, kernel, prefix, trace, units, unit in KERNELS:
        r = summarize(a.src, dst, a.round, name, kernel, prefix, trace, units, unit,
                      win.get(kernel) if trace == "trace" else None)
        print(name, json.dumps({k: v for k, v in (r or {}).items() if k != "pmc"}, indent=1))


if __name__ == "__main__":
    main()
