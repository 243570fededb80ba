"""A/B of the tiled encoder's grid (SCT_TUNE_ENCODE_GRID 0 resident / 1 one workgroup per tile)
on config 5's 1e9 x 28-bp reads, interleaved rounds, plus the outputs of both compared."""
import json
import sys

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import torch  # noqa: E402

import bench  # noqa: E402
from sctools_amd import _lib, synthetic  # noqa: E402

dev = torch.device("cuda", 0)
n, L = synthetic.CONFIG5_READS, synthetic.CONFIG5_READ_LENGTH
g = torch.Generator(device=dev).manual_seed(5)
seqs = torch.randint(0, 4, (n, L), dtype=torch.uint8, device=dev, generator=g)
for r0 in range(0, n, 50_000_000):
    x = seqs[r0:r0 + 50_000_000]
    x.copy_(65 + 2 * x + 15 * (x == 2).to(torch.uint8))
if __import__("os").environ.get("WITH_N"):  # 1 % of the reads with one N, as bench.path_config5_encode
    nrows = torch.arange(0, n, 100, device=dev)
    seqs[nrows, torch.randint(0, L, (nrows.numel(),), device=dev, generator=g)] = ord("N")
out = {k: torch.empty(n, dtype=t, device=dev) for k, t in (("c0", torch.int64), ("c1", torch.int64),
                                                            ("g", torch.uint8), ("f", torch.uint8))}
lib = _lib.lib()
stream = torch.cuda.current_stream(dev).cuda_stream
res = {0: [], 1: []}
for rnd in range(3):
    for mode in (0, 1):
        with _lib.tuning(encode_grid=mode):
            c = out["c%d" % mode]
            res[mode].append(bench._events_ms(lambda: _lib.check(lib.sct_encode(
                2, seqs.data_ptr(), n, L, L, c.data_ptr(), out["g"].data_ptr(), out["f"].data_ptr(), stream)), 3, dev))
torch.cuda.synchronize()
same = bool(torch.equal(out["c0"], out["c1"]))
print(json.dumps({"resident_ms": res[0], "onepass_ms": res[1], "outputs_equal": same,
                  "tbps": {k: n * (L + 10) / (min(v) * 1e-3) / 1e12 for k, v in res.items()}}))
