"""Benchmark: Hamming pair-comparisons/s, 737,280-barcode all-pairs histogram (BASELINE.json).

One step = the whole hot path of Barcodes.summarize_hamming_distances on device-
resident codes, with the count scheme the library picks (AUTO; --scheme forces one):
build the plan's tables, count this rank's share of the work items, all-reduce the
counts over RCCL (N > 1), copy them to the host, invert them to the exact histogram
and compute the numpy-exact summary.  At 737K 16-bp codes AUTO is SPECTRAL (the
Walsh-Hadamard route, DESIGN.md §3.8: no pair is enumerated, the histogram is the same
bit for bit); the pair-enumerating MOMENTS kernel is timed beside it as `pair_kernel`.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)

Rank 0 prints one JSON line.  `value` = all pairs of the whole job / max-over-ranks
wall time of the K timed steps.  `roofline` prices the dominant kernel over its average
duration, measured with HIP events on the stream it runs on: SPECTRAL's tile kernel
with its algorithmic int32 ops (14 butterfly add/subs + 1 square-accumulate per
transform value), or the pair count kernel with SURVEY.md §8(d)'s 4 ops per 16-bp pair.  `cpu_baseline` times the C oracle restatement (test infrastructure,
never the product) on a bounded row sample of the same workload, rank 0 only.
"""

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from sctools_amd import _lib, sharding, synthetic  # noqa: E402

# Full-rate VALU issue: 256 CU x 4 SIMD32 x 32 lanes/clk x 2.4 GHz = 78.6 Tops/s (2-source
# int32 ops; measured 121 lane-ops/clk/CU for v_xor_b32 by tools/valu_peak.hip / valu_banks.hip).
VALU_PEAK_OPS = 256 * 128 * 2.4e9
HBM_PEAK_BPS = 8.0e12  # MI355X HBM3E (MI355X_MICROARCH.md)
ALGO_OPS_PER_PAIR = 4  # XOR, shift-OR, AND, popcount per 32-bit code word
# VALU issue slots the bit-sliced count kernel spends per pair at 16 bp, from its unmasked
# loop (v_bcnt_u32_b32 counts 2: half rate on gfx950), per count scheme:
#   SUBSETS (nibble tables, full unroll): 33 v_bitop3 + 16 v_bcnt + 6 v_xor/v_and per 32 pairs;
#   MOMENTS (triple tables, unroll 1): 24 v_bitop3 + 13 v_bcnt + 4 v_xor/v_and + 3 v_add.
ISSUE_SLOTS_PER_PAIR = {_lib.SCHEME_SUBSETS: (33 + 2 * 16 + 6) / 32.0,
                        _lib.SCHEME_MOMENTS: (24 + 2 * 13 + 4 + 3) / 32.0}
# SPECTRAL tile kernel: per slice of 2^14 transform values, 14 butterfly levels (one add
# or sub per value per level) and one square-accumulate per value
SPECTRAL_OPS_PER_SLICE = (1 << 14) * (14 + 1)
SCHEMES = {"auto": _lib.SCHEME_AUTO, "subsets": _lib.SCHEME_SUBSETS, "moments": _lib.SCHEME_MOMENTS,
           "spectral": _lib.SCHEME_SPECTRAL}
SCHEME_NAMES = {v: k for k, v in SCHEMES.items()}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=2, choices=[1, 2, 5])
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU baseline sample time")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend (nccl = RCCL)")
    ap.add_argument("--scheme", default="auto", choices=sorted(SCHEMES))
    ap.add_argument("--pair-steps", type=int, default=5,
                    help="steps of the pair-enumerating MOMENTS kernel timed beside SPECTRAL (N=1)")
    return ap.parse_args()


def cpu_baseline(codes, target_s):
    """C oracle (OpenMP popcount restatement of encodings.py:113-121) on rows [0, R)."""
    from oracle import oracle as O
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    n = codes.size
    lib = O.c_oracle()
    # calibrate on a ~0.5 s sample, then size the sample to ~target_s
    rows = 256
    while True:
        t = time.perf_counter()
        O.c_hist_rows(codes, 0, rows, threads=threads)
        dt = time.perf_counter() - t
        if dt > 0.5 or rows >= n // 4:
            break
        rows *= 4
    rows = int(min(n - 1, max(rows, rows * target_s / dt)))
    t = time.perf_counter()
    O.c_hist_rows(codes, 0, rows, threads=threads)
    dt = time.perf_counter() - t
    pairs = rows * (n - 1) - rows * (rows - 1) // 2
    # the scalar loop itself (1 core), short sample
    srow = 64
    t = time.perf_counter()
    O.c_hist_rows(codes, 0, srow, scalar=True)
    sdt = time.perf_counter() - t
    spairs = srow * (n - 1) - srow * (srow - 1) // 2
    return {"value": pairs / dt, "unit": "pairs/s", "cores": lib.oracle_threads() if threads == 0 else threads,
            "kind": "port",
            "sample": "C oracle popcount (oracle/sct_oracle.c) over rows [0,%d) of the same %d-code set: "
                      "%d pairs in %.2f s" % (rows, n, pairs, dt),
            "scalar_1core_pairs_per_s": spairs / sdt,
            "python_reference_1core_pairs_per_s": 752540.0}


def _traffic(name):
    """HBM bytes per launch of the kernel from the committed PMC summary (FETCH_SIZE +
    WRITE_SIZE, gfx950-corrected; tools/summarize_profile.py), or None."""
    pmc = os.path.join(ROOT, "profiles", name)
    if os.path.exists(pmc):
        with open(pmc) as f:
            return json.load(f).get("hbm_bytes_per_launch")
    return None


def spectral_roofline(tk, step_count_ms, my_slices):
    """SPECTRAL's two kernels per chunk: seed (writes 2^14 int8 values per slice) and tile
    (reads them back: 14-bit WHT on the matrix cores + F^2 binning).  Both move 16 KiB per
    slice through HBM, so the roofline is HBM bandwidth; the dominant (slower) kernel is the
    one reported, the other beside it."""
    per_launch = tk["units"]
    launches = -(-my_slices // per_launch)
    algo_bytes = per_launch * (1 << 14)  # int8 seed values per launch (seed writes, tile reads)
    kern = {"tile": {"kernel": "sct_spectral::tile_mfma2_pf_kernel (int8 seeds)", "ms": tk["kernel_ms"],
                     "traffic": _traffic("pmc_spectral_latest.json")},
            "seed": {"kernel": "sct_spectral::seed_kernel<int8_t>", "ms": tk["seed_ms"],
                     "traffic": _traffic("pmc_spectral_seed_latest.json")}}
    for k in kern.values():
        k["achieved_gbs"] = algo_bytes / (k["ms"] * 1e-3) / 1e9
        k["frac"] = k["achieved_gbs"] * 1e9 / HBM_PEAK_BPS
    dom, other = ("seed", "tile") if tk["seed_ms"] >= tk["kernel_ms"] else ("tile", "seed")
    d = kern[dom]
    tile_ops = per_launch * SPECTRAL_OPS_PER_SLICE / (tk["kernel_ms"] * 1e-3)
    return {"bound": "hbm", "achieved": d["achieved_gbs"], "peak": HBM_PEAK_BPS / 1e9, "unit": "GB/s",
            "frac": d["frac"], "traffic": d["traffic"], "kernel": d["kernel"], "kernel_ms": d["ms"],
            "other_kernel": dict(kern[other], name=other),
            "slices_per_launch": per_launch, "launches_per_step": launches,
            "algo_bytes_per_launch": algo_bytes,
            "count_ms_per_step": step_count_ms,
            "chunk_frac": 2 * algo_bytes / ((tk["seed_ms"] + tk["kernel_ms"]) * 1e-3) / HBM_PEAK_BPS,
            "tile_valu_equivalent": {"algo_ops_per_slice": SPECTRAL_OPS_PER_SLICE, "achieved_tops": tile_ops / 1e12,
                                     "peak_tops": VALU_PEAK_OPS / 1e12, "frac": tile_ops / VALU_PEAK_OPS,
                                     "note": "14 butterfly add/subs + 1 square-accumulate per value as int32 "
                                             "VALU ops; 12 of the 14 levels run on the matrix cores"},
            "note": "kernel_ms: HIP events around 5 back-to-back launches of each kernel on the bench "
                    "stream; algo bytes = the int8 seed values of one launch (the seed kernel writes them, "
                    "the tile kernel reads them); traffic: HBM bytes per launch from PMC "
                    "(tools/summarize_profile.py); chunk_frac = both kernels' bytes over their summed time"}


def pair_roofline(plan, my_pairs, kms, L, moments_ms):
    achieved = my_pairs * ALGO_OPS_PER_PAIR / (kms * 1e-3)
    slots_per_pair = ISSUE_SLOTS_PER_PAIR[plan.scheme] if L == 16 else float("nan")
    slots = my_pairs * slots_per_pair / (kms * 1e-3)
    return {"bound": "valu", "achieved": achieved / 1e12, "peak": VALU_PEAK_OPS / 1e12,
            "unit": "Tops/s", "frac": achieved / VALU_PEAK_OPS, "traffic": _traffic("pmc_allpairs_latest.json"),
            "kernel": "allpairs_count_kernel<8>", "kernel_ms": kms,
            "algo_ops_per_pair": ALGO_OPS_PER_PAIR,
            "issue_slots_per_pair": slots_per_pair,
            "scheme": SCHEME_NAMES[plan.scheme],
            "moments_ms": moments_ms,
            "issue_slot_frac": slots / VALU_PEAK_OPS,
            "note": "frac > 1: the bit-sliced kernel needs %.2f VALU issue slots per "
                    "pair where SURVEY 8(d)'s formulation needs 4 ops (5 slots: "
                    "v_bcnt is half rate); issue_slot_frac is the VALU utilisation" % slots_per_pair}


def time_pair_kernel(d_codes, n, L, pairs_total, steps):
    """The pair-enumerating MOMENTS kernel on the same codes (whole step: build, moments,
    count, inversion), for comparison with SPECTRAL."""
    plan = _lib.AllPairsPlan(d_codes.data_ptr(), n, 2 * L, scheme=_lib.SCHEME_MOMENTS)
    dev = d_codes.device
    counts = torch.zeros(plan.ncounts, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    kms, hist = [], None
    for i in range(steps + 1):
        if i == 1:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        counts.zero_()
        plan.build(s.cuda_stream)
        plan.moments(counts.data_ptr(), 0, 1, s.cuda_stream)
        ev0.record(s)
        plan.count(counts.data_ptr(), 0, plan.items, 0, s.cuda_stream)
        ev1.record(s)
        hist = sharding.combine_counts(counts, None, plan.scheme, plan.nbins)
        if i:
            kms.append(ev0.elapsed_time(ev1))
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    plan.close()
    assert int(hist.sum()) == pairs_total
    km = float(np.mean(kms))
    return {"scheme": "moments", "value": pairs_total / dt, "unit": "pairs/s", "ms_per_step": dt * 1e3,
            "steps": steps, "kernel_ms": km,
            "kernel_frac": pairs_total * ALGO_OPS_PER_PAIR / (km * 1e-3) / VALU_PEAK_OPS}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # one process per GPU; more ranks than GPUs (a rehearsal on a 1-GPU box) share them
        local_dev = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local_dev)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_dev))
        else:
            dist.init_process_group(args.backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    _lib.check(_lib.lib().sct_set_device(dev.index))

    n, L, seed = synthetic.CONFIGS[args.config]
    codes = synthetic.whitelist_codes(n, L, seed)
    d_codes = torch.from_numpy(codes.view(np.int64)).to(dev)
    plan = _lib.AllPairsPlan(d_codes.data_ptr(), n, 2 * L, scheme=SCHEMES[args.scheme])
    spectral = plan.scheme == _lib.SCHEME_SPECTRAL
    b, e = sharding.item_range(plan.items, rank, world)
    counts = torch.zeros(plan.ncounts, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    kernel_ms = []

    # the moments pass (independent of the table) runs on a side stream beside the build
    side = torch.cuda.Stream(dev)
    ev_zero, ev_mom = torch.cuda.Event(), torch.cuda.Event()
    evm0, evm1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    moments_ms = []

    def step(record):
        counts.zero_()
        ev_zero.record(stream)
        side.wait_event(ev_zero)
        if record:
            evm0.record(side)
        plan.moments(counts.data_ptr(), rank, world, side.cuda_stream)  # this rank's share
        if record:
            evm1.record(side)
        ev_mom.record(side)
        plan.build(sptr, b, e)  # sort + the selection-table chunks this rank's items read
        stream.wait_event(ev_mom)  # the count kernel runs alone (its timing stays clean)
        if record:
            ev0.record(stream)
        plan.count(counts.data_ptr(), b, e, 0, sptr)
        if record:
            ev1.record(stream)
        # RCCL all-reduce (N > 1), D2H, exact inversion
        hist = sharding.combine_counts(counts, None, plan.scheme, plan.nbins)
        if record:
            kernel_ms.append(ev0.elapsed_time(ev1))
            moments_ms.append(evm0.elapsed_time(evm1))
        return hist, _lib.summary_from_hist(hist)

    for _ in range(args.warmup):
        hist, summ = step(False)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        hist, summ = step(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    pairs_total = plan.pairs
    assert int(hist.sum()) == pairs_total, "histogram does not cover every pair"
    my_pairs = plan.range_pairs(b, e)
    kms = float(np.mean(kernel_ms))
    if spectral:
        # the tile / seed kernels apart: back-to-back launches between HIP events on `stream`
        scratch = torch.zeros(plan.ncounts, dtype=torch.int64, device=dev)
        tk = plan.time_kernels(scratch.data_ptr(), b, e, 5, sptr)
        roofline = spectral_roofline(tk, kms, plan.items // world)
    else:
        roofline = pair_roofline(plan, my_pairs, kms, L, float(np.mean(moments_ms)))
    pair_kernel = None
    if spectral and world == 1 and args.pair_steps > 0:
        pair_kernel = time_pair_kernel(d_codes, n, L, pairs_total, args.pair_steps)

    if rank == 0:
        out = {
            "metric": "Hamming pair-comparisons/sec, 737K 10x whitelist all-pairs, 1-8 GPUs",
            "value": pairs_total * args.steps / elapsed,
            "unit": "pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "i32" if spectral else "u32",
            "data": "synthetic (seeded uniform random unique 16-bp codes, sctools_amd/synthetic.py)",
            "config": {"workload": "config %d: %d-barcode all-pairs TwoBit Hamming histogram + summary"
                                   % (args.config, n),
                       "barcodes": n, "barcode_length": L, "pairs": pairs_total,
                       "scheme": SCHEME_NAMES[plan.scheme],
                       "parallelism": ("transform-slice shards" if spectral else "item-range + moment shards")
                       + ", RCCL all-reduce of %d counts" % plan.ncounts if world > 1 else "single GPU"},
            "roofline": roofline,
            "summary": dict(zip(("minimum", "p25", "median", "p75", "maximum", "average"),
                                [float(x) for x in summ])),
        }
        if pair_kernel is not None:
            out["pair_kernel"] = pair_kernel
        if not args.no_cpu and world == 1:
            out["cpu_baseline"] = cpu_baseline(codes, args.cpu_seconds)
        print(json.dumps(out), flush=True)
    plan.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
