"""(Needs the parted build of commit history: the SCT_TUNE_FASTQ_PARTS knob was removed after this
A/B, profiles/ab_fastq_parts_r06.jsonl.)  The fused FASTQ extraction (bench.py path_fastq: 20M device-resident records) with its count
passes overlapped part by part (the default) against one count pass first (fastq_parts=1), rounds
interleaved on one box.  One JSON line per run, then a summary."""
import json
import sys

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import torch  # noqa: E402

import bench  # noqa: E402
from sctools_amd import _lib  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
copy = bench.copy_ceiling_gbs(dev)
res = {}
for rnd in range(3):
    for name, parts in (("parts1", 1), ("default", None), ("parts2", 2), ("parts8", 8)):
        with _lib.tuning(fastq_parts=parts):
            r = bench.path_fastq(dev, 7, copy)
        res.setdefault(name, []).append(r["ms"])
        print(json.dumps({"variant": name, "round": rnd, "ms": r["ms"], "check": r.get("check")}), flush=True)
print(json.dumps({"summary": {k: sorted(v)[1] for k, v in res.items()}}))
