"""Ablation timing of sct_fastq_extract_fused on bench.path_fastq's 20M-record FASTQ: the shipped
library and the SCT_FQ_ABL builds of tools/build_fq_abl.sh (1 no per-tile items, 2 name checks
only, 3 no CB encode, 4 no terminator list), each in its own process (SCTOOLS_HIP_LIB), rounds
interleaved.  Ablation results are wrong by design; only the time is read."""
import json
import os
import subprocess
import sys

ROOT = __file__.rsplit("/tools/", 1)[0]
if os.environ.get("FQ_CHILD"):
    sys.path.insert(0, ROOT)
    import torch
    import bench
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    if os.environ.get("FQ_PATH") == "pipeline":  # FASTQ -> ThreeBit -> nearest (bench.path_pipeline)
        f = bench.path_pipeline(dev, 5, 6300.0, bench.host_threads()[0])
        print(json.dumps({"ms": f.get("ms"), "extract_ms": f.get("extract_ms"), "ok": f.get("error") is None}))
    else:
        f = bench.path_fastq(dev, 5, 6300.0)
        print(json.dumps({"ms": f.get("ms"), "ok": bool(f.get("check", {}).get("sampled"))}))
    sys.exit(0)
libs = {"base": None}  # the shipped library, then sctools_amd/libsctools_hip_<arg>.so per argument
for k in (sys.argv[1:] or ["fqabl1", "fqabl2", "fqabl3", "fqabl4"]):
    libs[k] = os.path.join(ROOT, "sctools_amd", "libsctools_hip_%s.so" % k)
res = {k: [] for k in libs}
for rnd in range(int(os.environ.get("ROUNDS", "2"))):
    for k, lib in libs.items():
        env = dict(os.environ, FQ_CHILD="1")
        if lib:
            env["SCTOOLS_HIP_LIB"] = lib
        out = subprocess.run([sys.executable, "-u", __file__], env=env, capture_output=True, text=True, timeout=180)
        if out.returncode != 0:
            print(out.stderr[-2000:], file=sys.stderr)
            sys.exit(out.returncode)
        r = json.loads(out.stdout.strip().splitlines()[-1])
        res[k].append(r)
        print(json.dumps({"lib": k, **r}), file=sys.stderr, flush=True)
print(json.dumps(res))
