"""bench.path_fastq under SCT_TUNE_FASTQ_ONEPASS = $FASTQ_MODE (for rocprofv3 passes of one form)."""
import json
import os
import sys

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import torch  # noqa: E402

import bench  # noqa: E402
from sctools_amd import _lib  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
with _lib.tuning(fastq_onepass=int(os.environ.get("FASTQ_MODE", "0"))):
    r = bench.path_fastq(dev, 3, 6300.0)
print(json.dumps({k: r.get(k) for k in ("ms", "check", "error")}))
