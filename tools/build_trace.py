"""The per-step plan build on its own (config 2's 737,280 codes, SPECTRAL): 50 builds back to back
on one stream, for a rocprofv3 kernel trace of the five build kernels and their launch gaps."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from sctools_amd import _lib, synthetic  # noqa: E402

n, L, seed = synthetic.CONFIGS[2]
codes = synthetic.whitelist_codes(n, L, seed)
d = torch.from_numpy(codes.astype("uint64").view("int64")).cuda()
plan = _lib.AllPairsPlan(d.data_ptr(), n, 2 * L, scheme=_lib.SCHEME_SPECTRAL)
s = torch.cuda.Stream()
for _ in range(50):
    plan.build(s.cuda_stream)
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record(s)
for _ in range(50):
    plan.build(s.cuda_stream)
b.record(s)
b.synchronize()
print("build ms (events, 50 back to back):", a.elapsed_time(b) / 50)
plan.close()
