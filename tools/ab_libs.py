"""Same-box A/B of bench.py side paths across library builds: each (library, knobs) variant in its
own process (SCTOOLS_HIP_LIB), rounds interleaved; one JSON line per run, then a summary.

  python tools/ab_libs.py --path whitelist --variant base=sctools_amd/libsctools_hip_base.so \
      --variant new= --variant nospec=:ingest_spec=0 [--rounds 3]

A variant is name=LIB[:knob=value,...]; an empty LIB is the working tree's library."""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def headline(dev, steps=20):
    """Config 2's pipelined step (ShardedAllPairs.run, what bench.py times) at W = 1 and for rank
    0's share at W = 8 (emulated: the rank's slice range, no all-reduce): ms per step."""
    import time
    import torch
    from sctools_amd import _lib, sharding, synthetic
    n, L, seed = synthetic.CONFIGS[2]
    codes = synthetic.whitelist_codes(n, L, seed)
    out = {}
    inv = _lib.counts_to_hist
    for world in (1, 8):
        with sharding.ShardedAllPairs(codes, 2 * L) as job:
            job.begin, job.end = sharding.item_range(job.plan.items, 0, world)
            _lib.counts_to_hist = inv if world == 1 else (lambda host, scheme, nbins: host)
            job.run(3)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            hists = job.run(steps)
            torch.cuda.synchronize()
            out["w%d_ms" % world] = (time.perf_counter() - t0) / steps * 1e3
            out["w%d_agree" % world] = all((h == hists[0]).all() for h in hists)
    _lib.counts_to_hist = inv
    return {"ms": out["w1_ms"], "ms_per_step": out, "check": {"steps_agree": out["w1_agree"] and out["w8_agree"]}}


def child(path, knobs):
    sys.path.insert(0, ROOT)
    import torch
    import bench
    from sctools_amd import _lib
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    copy = 6300.0
    threads = bench.host_threads()[0]
    fn = {"config4": lambda: bench.path_config4(dev, 5, copy, threads),
          "pipeline": lambda: bench.path_pipeline(dev, 5, copy, threads),
          "fastq": lambda: bench.path_fastq(dev, 5, copy),
          "whitelist": lambda: bench.path_whitelist(dev, 5, copy),
          "config5_allpairs": lambda: bench.path_config5_allpairs(dev, 5, copy),
          "dropin": lambda: bench.path_dropin(dev, 10, None),
          "headline": lambda: headline(dev)}[path]
    with _lib.tuning(**knobs):
        r = fn()
    keep = {k: r.get(k) for k in ("ms", "ms_per_step", "extract_ms", "query_ms", "index_build_ms", "check")}
    if path == "whitelist":
        keep = {"ms": r["whitelist_ingest"].get("ms"), "check": r["whitelist_ingest"].get("check"),
                "base_frequency_ms": r["base_frequency"].get("ms")}
    if path == "dropin":
        keep["breakdown_ms"] = r.get("breakdown_ms")
    if path == "config5_allpairs":
        keep["kernels"] = {"tile_ms": r["roofline"]["kernel_ms"], "seed_ms": r["roofline"]["other_kernel"]["ms"]}
    print(json.dumps(keep), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--path", default="config4")
    ap.add_argument("--variant", action="append", required=True)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--child", default=None)
    a = ap.parse_args()
    if a.child is not None:
        knobs = {}
        for kv in filter(None, a.child.split(",")):
            k, v = kv.split("=")
            knobs[k] = int(v)
        child(a.path, knobs)
        return
    variants = []
    for v in a.variant:
        name, rest = v.split("=", 1)
        lib, _, knobs = rest.partition(":")
        variants.append((name, lib, knobs))
    res = {name: [] for name, _, _ in variants}
    for rnd in range(a.rounds):
        for name, lib, knobs in variants:
            env = dict(os.environ)
            if lib:
                env["SCTOOLS_HIP_LIB"] = os.path.join(ROOT, lib)
            out = subprocess.run([sys.executable, "-u", __file__, "--path", a.path, "--variant", "x=", "--child", knobs],
                                 env=env, capture_output=True, text=True, timeout=300)
            if out.returncode != 0:
                print(json.dumps({"variant": name, "round": rnd, "rc": out.returncode, "err": out.stderr[-1500:]}),
                      flush=True)
                sys.exit(out.returncode if out.returncode > 0 else 1)
            r = json.loads(out.stdout.strip().splitlines()[-1])
            res[name].append(r)
            print(json.dumps({"variant": name, "round": rnd, **r}), flush=True)
    print(json.dumps({"summary": {k: [r.get("ms") or r.get("ms_per_step") for r in v] for k, v in res.items()}}))


if __name__ == "__main__":
    main()
