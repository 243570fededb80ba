"""A/B of sct_fastq_extract_fused's two forms (SCT_TUNE_FASTQ_ONEPASS: 0 = count pass, then the
extraction; 4 / 8 = one pass, a look-back over ranges of that many tiles) on bench.path_fastq's
20M-record FASTQ, interleaved rounds, each with the path's own correctness check."""
import json
import os
import sys

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import torch  # noqa: E402

import bench  # noqa: E402
from sctools_amd import _lib  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
modes = [int(x) for x in (sys.argv[1:] or ["0", "4", "8"])]
res = {m: {"ms": [], "ok": True} for m in modes}
for rnd in range(int(os.environ.get("ROUNDS", "3"))):
    for m in modes:
        with _lib.tuning(fastq_onepass=m):
            f = bench.path_fastq(dev, 3, 6300.0)
        res[m]["ms"].append(f.get("ms"))
        res[m]["ok"] = res[m]["ok"] and bool(f.get("check", {}).get("sampled"))
        print(json.dumps({"mode": m, "ms": f.get("ms"), "err": f.get("error")}), file=sys.stderr, flush=True)
print(json.dumps(res))
