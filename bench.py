"""Benchmark: Hamming pair-comparisons/s, 737,280-barcode all-pairs histogram (BASELINE.json).

One step = the whole hot path of Barcodes.summarize_hamming_distances on device-resident
codes, as one rank runs it (sctools_amd.sharding.ShardedAllPairs): build the plan's
tables, count this rank's share of the work items, all-reduce the counts over RCCL
(N > 1), copy them to the host, invert them to the exact histogram, then the numpy-exact
summary.  At 737K 16-bp codes the library's AUTO scheme is SPECTRAL (the Walsh-Hadamard
route): no pair is enumerated, yet the histogram of all P = n(n-1)/2
pair distances is exact, so `value` is PAIR-EQUIVALENT throughput (P / step time, cost
independent of n).  The K timed steps run pipelined two deep (ShardedAllPairs.run, two
plans): step k+1's build runs on its own stream beside step k's count, its count is queued
before the host waits for step k's all-reduce and histogram, and every step's histogram is
produced and checked (`ranks[].build_ms` is the build's overlapped span on its stream).  The pair-enumerating MOMENTS kernel is
timed beside it (N = 1) as `pair_kernel`.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2]

--gpus N > 1 without a launcher: bench.py itself starts N rank processes (one per GPU,
backend nccl = RCCL) before anything touches a GPU, and exits non-zero if fewer than N
GPUs are visible.  Under torchrun (WORLD_SIZE set) every process is one rank and
WORLD_SIZE must equal --gpus.  Rank 0 prints one JSON line: `value` = all pairs of the
whole job / max-over-ranks wall time of the K timed steps; `ranks` = per-rank count /
all-reduce / step times.  `roofline` prices the dominant kernel with HIP events on the
stream it runs on.  `cpu_baseline` (N = 1, rank 0) runs the C oracle restatement (test
infrastructure, never the product) on this host's cores and checks its histogram
against the GPU's.
"""

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Full-rate VALU issue: 256 CU x 4 SIMD x 32 lanes/clk x 2.4 GHz = 78.6 T lane-slots/s
# (measured 121 lane-ops/clk/CU for v_xor_b32, profiles/valu_peak_r01.json).
VALU_PEAK_OPS = 256 * 128 * 2.4e9
HBM_PEAK_BPS = 8.0e12  # MI355X HBM3E (MI355X_MICROARCH.md)
ALGO_OPS_PER_PAIR = 4  # XOR, shift-OR, AND, popcount per 32-bit code word
# SPECTRAL tile kernel: per slice of 2^14 transform values, 14 butterfly levels (one add
# or sub per value per level) and one square-accumulate per value
SPECTRAL_OPS_PER_SLICE = (1 << 14) * (14 + 1)
METRIC = "Hamming pair-comparisons/sec, 737K 10x whitelist all-pairs, 1-8 GPUs"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=2, choices=[1, 2, 5])
    ap.add_argument("--cpu-seconds", type=float, default=30.0,
                    help="CPU baseline budget: the whole job if it fits, else a row sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend (nccl = RCCL)")
    ap.add_argument("--scheme", default="auto", choices=["auto", "subsets", "moments", "spectral"])
    ap.add_argument("--pair-steps", type=int, default=5,
                    help="steps of the pair-enumerating MOMENTS kernel timed beside SPECTRAL (N=1)")
    ap.add_argument("--allow-shared-gpu", action="store_true",
                    help="rehearsal only: let more ranks than GPUs share devices")
    ap.add_argument("--stub", action="store_true",
                    help="launcher test: ranks form the group and all-reduce stub counts, no GPU")
    return ap.parse_args(argv)


# ------------------------------------------------------------------ launcher
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_local_ranks(args, argv):
    """Start args.gpus rank processes of this script (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*
    set, 127.0.0.1 rendezvous), stream their output, return the worst exit code.  Runs
    before this process touches a GPU (torch.cuda.device_count() does not initialise one)."""
    n = args.gpus
    if not args.stub and args.backend == "nccl" and not args.allow_shared_gpu:
        import torch
        vis = torch.cuda.device_count()
        if vis < n:
            print("bench.py: --gpus %d but only %d GPU(s) visible; refusing to time fewer ranks" % (n, vis),
                  file=sys.stderr, flush=True)
            return 2
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                code = p.poll()
                if code is None:
                    continue
                pending.remove(p)
                if code != 0:
                    rc = rc or (code if code > 0 else 128 - code)
                    for q in pending:  # one rank failed: the others would wait in a collective
                        q.send_signal(signal.SIGTERM)
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc


# ------------------------------------------------------------------ CPU baseline
def _host_info():
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
            if q != "max":
                quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": aff, "cgroup_cpu_quota": quota,
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS")}


def cpu_baseline(codes, gpu_hist, budget_s):
    """The C oracle (oracle/sct_oracle.c: encodings.py:113-121's popcount form over 32-bit
    AVX-512 lanes, OpenMP over rows) on every core this process may use: the whole job if it
    fits the budget (its histogram must equal the GPU's bin for bin), else rows [0, R)."""
    from oracle import oracle as O
    info = _host_info()
    # all host cores this job may use: OMP_NUM_THREADS when the box sets the CPU share,
    # else the affinity mask (nproc counts the whole machine on a shared box)
    threads = int(info["omp_num_threads_env"] or 0) or info["affinity_cpus"] or 1
    if info["cgroup_cpu_quota"]:
        threads = max(1, min(threads, int(round(info["cgroup_cpu_quota"]))))
    n = codes.size
    P = n * (n - 1) // 2
    rows = 2048
    t = time.perf_counter()
    _, simd = O.c_hist16(codes, 0, rows, threads=threads)
    dt = time.perf_counter() - t
    rate = (rows * (n - 1) - rows * (rows - 1) // 2) / dt
    out = {"unit": "pairs/s", "cores": threads, "kind": "port", **info,
           "kernel": "oracle_hist16 (AVX-512 VPOPCNTDQ)" if simd else "oracle_hist_popcnt (scalar popcnt)"}
    if P / rate <= budget_s:
        t = time.perf_counter()
        hist, _ = O.c_hist16(codes, threads=threads)
        dt = time.perf_counter() - t
        out.update(value=P / dt, sample="the whole job: all %d pairs of the same %d-code set in %.2f s" % (P, n, dt),
                   hist_match=bool(hist[:gpu_hist.size].tolist() == [int(x) for x in gpu_hist]
                                   and not hist[gpu_hist.size:].any()))
    else:
        rows = int(min(n - 1, max(rows, rows * budget_s / (dt * 1.2))))
        t = time.perf_counter()
        O.c_hist16(codes, 0, rows, threads=threads)
        dt = time.perf_counter() - t
        pairs = rows * (n - 1) - rows * (rows - 1) // 2
        out.update(value=pairs / dt, sample="rows [0,%d) of the same %d-code set: %d pairs in %.2f s"
                   % (rows, n, pairs, dt), hist_match=None)
    srow = 48  # the statement-for-statement loop of encodings.py:113-121, 1 core
    t = time.perf_counter()
    O.c_hist_rows(codes, 0, srow, scalar=True)
    sdt = time.perf_counter() - t
    out["scalar_1core_pairs_per_s"] = (srow * (n - 1) - srow * (srow - 1) // 2) / sdt
    out["python_reference_1core_pairs_per_s"] = 752540.0  # SURVEY.md §6, measured in the build container
    return out


# ------------------------------------------------------------------ rooflines
def _traffic(name):
    """HBM bytes per launch of the kernel from the committed PMC summary, or None."""
    pmc = os.path.join(ROOT, "profiles", name)
    if os.path.exists(pmc):
        with open(pmc) as f:
            return json.load(f).get("hbm_bytes_per_launch")
    return None


def spectral_roofline(tk, step_count_ms, my_slices):
    """SPECTRAL's two kernels per chunk: seed (writes 2^14 int8 values per slice) and tile
    (reads them back: 14-bit WHT on the matrix cores + F^2 binning).  Both move 16 KiB per
    slice through HBM, so the roofline is HBM bandwidth; the slower kernel is reported."""
    per_launch = tk["units"]
    launches = -(-my_slices // per_launch)
    algo_bytes = per_launch * (1 << 14)
    kern = {"tile": {"kernel": "sct_spectral::tile_reg_p16_kernel (int8 seeds)", "ms": tk["kernel_ms"],
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


def issue_slots_per_pair(scheme):
    """VALU issue slots the bit-sliced count kernel spends per 16-bp pair, from its
    unmasked loop (v_bcnt_u32_b32 is half rate on gfx950: 2 slots)."""
    from sctools_amd import _lib
    return {_lib.SCHEME_SUBSETS: (33 + 2 * 16 + 6) / 32.0,     # nibble tables, full unroll
            _lib.SCHEME_MOMENTS: (24 + 2 * 13 + 4 + 3) / 32.0}.get(scheme, float("nan"))


def pair_roofline(job, my_pairs, kms, L):
    achieved = my_pairs * ALGO_OPS_PER_PAIR / (kms * 1e-3)
    spp = issue_slots_per_pair(job.scheme) if L == 16 else float("nan")
    slots = my_pairs * spp / (kms * 1e-3)
    t = job.timings()
    return {"bound": "valu", "achieved": achieved / 1e12, "peak": VALU_PEAK_OPS / 1e12,
            "unit": "Tops/s", "frac": achieved / VALU_PEAK_OPS, "traffic": _traffic("pmc_allpairs_latest.json"),
            "kernel": "allpairs_count_kernel<8>", "kernel_ms": kms, "algo_ops_per_pair": ALGO_OPS_PER_PAIR,
            "issue_slots_per_pair": spp, "moments_ms": t["moments_ms"], "issue_slot_frac": slots / VALU_PEAK_OPS,
            "note": "frac > 1: the bit-sliced kernel needs %.2f VALU issue slots per pair where SURVEY "
                    "8(d)'s formulation needs 4 ops; issue_slot_frac is the VALU utilisation" % spp}


def time_pair_kernel(d_codes, L, steps):
    """The pair-enumerating MOMENTS kernel on the same codes (whole step: build, moments,
    count, inversion), for comparison with SPECTRAL."""
    import torch
    from sctools_amd import _lib, sharding
    with sharding.ShardedAllPairs(d_codes, 2 * L, _lib.SCHEME_MOMENTS) as job:
        hist = job.step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            hist = job.step(timing=True)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        P = job.plan.pairs
        assert int(hist.sum()) == P
        kms = job.timings()["count_ms"]
        spp = issue_slots_per_pair(job.scheme)
        return {"scheme": "moments", "value": P / dt, "unit": "pairs/s", "ms_per_step": dt * 1e3, "steps": steps,
                "kernel_ms": kms, "kernel_frac": P * ALGO_OPS_PER_PAIR / (kms * 1e-3) / VALU_PEAK_OPS,
                "issue_slots_per_pair": spp,
                "issue_slot_frac": P * spp / (kms * 1e-3) / VALU_PEAK_OPS,
                "note": "kernel_frac counts SURVEY 8(d)'s 4 ops per pair and exceeds 1 because the kernel "
                        "is bit-sliced; issue_slot_frac is the fraction of the VALU issue slots it uses"}


# ------------------------------------------------------------------ ranks
def run_stub(args, rank, world):
    """Launcher check without a GPU: the ranks form a gloo group and all-reduce stub counts
    (rank r contributes (r + 1) * [0, 1, ..., 17]) `steps` times."""
    import torch
    import torch.distributed as dist
    dist.init_process_group(args.backend, rank=rank, world_size=world)
    try:
        base = torch.arange(18, dtype=torch.int64)
        want = base * (world * (world + 1) // 2)
        ok = True
        t0 = time.perf_counter()
        for _ in range(args.warmup + args.steps):
            c = base * (rank + 1)
            dist.all_reduce(c)
            ok = ok and torch.equal(c, want)
        dt = time.perf_counter() - t0
        flags = torch.tensor([int(ok), rank], dtype=torch.int64)
        allf = [torch.zeros_like(flags) for _ in range(world)]
        dist.all_gather(allf, flags)
        if rank == 0:
            print(json.dumps({"stub": True, "n_gpus": dist.get_world_size(), "backend": dist.get_backend(),
                              "ranks_seen": sorted(int(f[1]) for f in allf),
                              "allreduce_ok": all(int(f[0]) for f in allf), "steps": args.steps,
                              "warmup": args.warmup, "seconds": dt}), flush=True)
    finally:
        dist.destroy_process_group()
    return 0


def run_rank(args, rank, world, local):
    import torch
    import torch.distributed as dist
    from sctools_amd import _lib, sharding, synthetic

    ndev = torch.cuda.device_count()
    if local >= ndev and not args.allow_shared_gpu:
        print("bench.py: rank %d (local %d) has no GPU of its own (%d visible)" % (rank, local, ndev),
              file=sys.stderr, flush=True)
        return 2
    dev_index = local % max(1, ndev)
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        else:
            dist.init_process_group(args.backend, rank=rank, world_size=world)
    backend = dist.get_backend() if world > 1 else None
    _lib.check(_lib.lib().sct_set_device(dev_index))

    n, L, seed = synthetic.CONFIGS[args.config]
    codes = synthetic.whitelist_codes(n, L, seed)
    scheme = {"auto": _lib.SCHEME_AUTO, "subsets": _lib.SCHEME_SUBSETS, "moments": _lib.SCHEME_MOMENTS,
              "spectral": _lib.SCHEME_SPECTRAL}[args.scheme]
    job = sharding.ShardedAllPairs(codes, 2 * L, scheme)
    spectral = job.scheme == _lib.SCHEME_SPECTRAL
    # steps run software-pipelined two deep (ShardedAllPairs.run): every step's zero, build,
    # count, all-reduce, read-back and inversion happen inside the timed region; step k+1's
    # kernels are queued before the host waits for step k's histogram
    job.run(args.warmup)
    job.reset_timings()  # the timings cover the timed steps only
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    hists = job.run(args.steps, timing=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    mine = time.perf_counter() - t0  # this rank's own wall time (before the max)
    tm = job.timings()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        row = torch.tensor([rank, tm["count_ms"], tm["allreduce_us"], tm["build_ms"], mine * 1e3 / args.steps,
                            job.end - job.begin], dtype=torch.float64, device=dev)
        rows = [torch.zeros_like(row) for _ in range(world)]
        dist.all_gather(rows, row)
        per_rank = [dict(zip(("rank", "count_ms", "allreduce_us", "build_ms", "step_ms", "items"),
                             [float(v) for v in r.cpu().tolist()])) for r in rows]
    else:
        per_rank = [{"rank": 0, "count_ms": tm["count_ms"], "allreduce_us": None, "build_ms": tm["build_ms"],
                     "step_ms": mine * 1e3 / args.steps, "items": job.end - job.begin}]
    for r in per_rank:
        r["rank"], r["items"] = int(r["rank"]), int(r["items"])

    hist = hists[-1]
    assert len(hists) == args.steps and all(np.array_equal(h, hist) for h in hists), "steps disagree"
    P = job.plan.pairs
    assert int(hist.sum()) == P, "histogram does not cover every pair"
    summ = _lib.summary_from_hist(hist)
    stream = torch.cuda.current_stream(dev).cuda_stream
    if spectral:  # the tile / seed kernels apart: back-to-back launches between HIP events
        scratch = torch.zeros(job.plan.ncounts, dtype=torch.int64, device=dev)
        tk = job.plan.time_kernels(scratch.data_ptr(), job.begin, job.end, 5, stream)
        roofline = spectral_roofline(tk, tm["count_ms"], job.end - job.begin)
    else:
        roofline = pair_roofline(job, job.my_pairs(), tm["count_ms"], L)
    pair_kernel = None
    if spectral and world == 1 and args.pair_steps > 0:
        pair_kernel = time_pair_kernel(job.d_codes, L, args.pair_steps)
    job.close()

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": P * args.steps / elapsed,
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
                       "barcodes": n, "barcode_length": L, "pairs": P,
                       "scheme": {0: "subsets", 1: "moments", 2: "spectral"}[job.scheme],
                       "value_kind": ("pair-equivalent: the exact histogram of all P pairs from a Walsh-Hadamard "
                                      "transform that enumerates no pair (cost independent of n)") if spectral
                       else "enumerated pairs",
                       "parallelism": ("%d ranks, %s; %s all-reduce of %d int64 counts" % (
                           world, "transform-slice shards" if spectral else "item-range + moment shards",
                           "RCCL" if backend == "nccl" else str(backend), job.plan.ncounts))
                       if world > 1 else "single GPU",
                       "backend": backend},
            "ranks": per_rank,
            "roofline": roofline,
            "summary": dict(zip(("minimum", "p25", "median", "p75", "maximum", "average"),
                                [float(x) for x in summ])),
            "hist": [int(x) for x in hist],
        }
        if pair_kernel is not None:
            out["pair_kernel"] = pair_kernel
        if not args.no_cpu and world == 1:
            out["cpu_baseline"] = cpu_baseline(codes, hist, args.cpu_seconds)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        if args.gpus > 1:
            return launch_local_ranks(args, argv)
        world, rank, local = 1, 0, 0
    else:
        world = int(env_world)
        rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", str(rank)))
        if world != args.gpus:
            print("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world), file=sys.stderr, flush=True)
            return 2
    if args.stub:
        return run_stub(args, rank, world)
    return run_rank(args, rank, world, local)


if __name__ == "__main__":
    sys.exit(main())
