"""A/B of the ingest extraction's tiles per workgroup (SCT_TUNE_INGEST_TILES; 0 = contiguous
ranges over the resident grid) on the whitelist and FASTQ bench paths, interleaved rounds; each
path's own correctness check is kept for every setting."""
import json
import sys

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import torch  # noqa: E402

import bench  # noqa: E402
from sctools_amd import _lib  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
copy = 6300.0
settings = [int(x) for x in (sys.argv[1:] or ["0", "1", "2", "4", "16", "64"])]
res = {k: {"wl_ms": [], "fq_ms": [], "ok": True} for k in settings}
for rnd in range(int(__import__("os").environ.get("ROUNDS", "2"))):
    for k in settings:
        with _lib.tuning(ingest_tiles=k):
            w = bench.path_whitelist(dev, 5, copy)["whitelist_ingest"]
            f = bench.path_fastq(dev, 3, copy)
        res[k]["wl_ms"].append(w["ms"])
        res[k]["fq_ms"].append(f["ms"])
        res[k]["ok"] = res[k]["ok"] and w["check"]["every_line"] and f["check"]["sampled"]
        print(json.dumps({"tiles": k, "wl": w["ms"], "fq": f["ms"]}), file=sys.stderr, flush=True)
print(json.dumps(res))
