"""Where the drop-in FASTQ -> nearest flow (bench.path_fastq_stream_to_nearest) spends its time:
the file pieces split into the read / carry-over in Python, the C chunk call (staging copies, H2D,
index, extraction) and the fetch (D2H), then ThreeBit.encode_array and the WhitelistCorrector build and queries, each
wrapped with a wall-clock timer.  One JSON line.  (GPU box; writes a 1.38 GB file under /tmp.)
--no-stage: the next piece is not copied ahead (FastqStream.stage a no-op), to see what the
caller's copies pay for sharing the link with it."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from sctools_amd import _lib, barcode, encodings  # noqa: E402

T = {}


def wrap(obj, name, key):
    fn = getattr(obj, name)

    def timed(*a, **k):
        t = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            T[key] = T.get(key, 0.0) + time.perf_counter() - t
    setattr(obj, name, timed)


if "--no-stage" in sys.argv:
    _lib.FastqStream.stage = lambda self, *a, **k: None
wrap(_lib.FastqStream, "chunk", "stream.chunk (C chunk + fetch)")
wrap(_lib.lib(), "sct_fastq_stream_chunk", "  sct_fastq_stream_chunk")
wrap(_lib.lib(), "sct_fastq_stream_fetch", "  sct_fastq_stream_fetch")
wrap(encodings.ThreeBit, "encode_array", "ThreeBit.encode_array")
wrap(_lib, "encode_stream", "  _lib.encode_stream")
wrap(barcode.WhitelistCorrector, "__init__", "WhitelistCorrector (index build)")
wrap(barcode.WhitelistCorrector, "nearest", "WhitelistCorrector.nearest")
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
r = bench.path_fastq_stream_to_nearest(dev, bench.host_threads()[0])
T = {k: v for k, v in T.items()}  # both runs (warm + timed): halve for one
print(json.dumps({"no_stage": "--no-stage" in sys.argv, "flow_ms": r.get("ms"), "breakdown_ms": r.get("breakdown_ms"),
                  "wrapped_ms_two_runs": {k: v * 1e3 for k, v in T.items()}, "check": r.get("check")}))
