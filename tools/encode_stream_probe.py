"""sct_encode_stream_host on one FASTQ-flow piece (3.3M page-locked 16-base rows, ThreeBit): wall
time per call for several chunk sizes (0 = the default split), against the bare H2D + D2H copies of
the same bytes timed alone.  One JSON line."""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from sctools_amd import _lib  # noqa: E402

n, L = 3_300_000, 16
rows = _lib.pinned.empty((n, L), np.uint8)
rows[:] = np.frombuffer(b"ACGT", np.uint8)[np.random.default_rng(1).integers(0, 4, (n, L))]
out = {}
for chunk in (0, 1 << 19, 1 << 20, 1 << 21, n):
    ts = []
    for _ in range(7):
        t = time.perf_counter()
        codes, gc, flags = _lib.encode_stream(3, rows, chunk)
        ts.append((time.perf_counter() - t) * 1e3)
    out["chunk_%d" % chunk] = float(np.median(ts[2:]))
dev = torch.device("cuda", 0)
d_in = torch.empty(n * L, dtype=torch.uint8, device=dev)
d_out = torch.empty(n * 10, dtype=torch.uint8, device=dev)
h_in = torch.from_numpy(rows.reshape(-1))
h_out = torch.from_numpy(_lib.pinned.empty(n * 10, np.uint8))
ts = []
for _ in range(7):
    torch.cuda.synchronize()
    t = time.perf_counter()
    d_in.copy_(h_in, non_blocking=True)
    h_out.copy_(d_out, non_blocking=True)
    torch.cuda.synchronize()
    ts.append((time.perf_counter() - t) * 1e3)
out["copies_only"] = float(np.median(ts[2:]))
out["pinned_in"] = _lib.host_pinned(rows)
print(json.dumps(out))
