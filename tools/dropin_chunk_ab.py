"""The default (workspace-freeing) drop-in call at several SPECTRAL chunk sizes: each chunk of
2^k slices needs a 2^(k+14)-byte intermediate that the call maps and unmaps, so a smaller chunk maps
less but launches the seed / tile pair more often.  Barcodes(dict of config 2).summarize_hamming_
distances(), wall-clock medians, rounds interleaved; keep_workspace(True) beside for reference."""
import json
import sys
import time

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import torch  # noqa: E402

from sctools_amd import _lib, barcode, synthetic  # noqa: E402

n, L, seed = synthetic.CONFIGS[2]
codes = synthetic.whitelist_codes(n, L, seed)
b = barcode.Barcodes(dict.fromkeys((int(c) for c in codes), 1), L)
ref = b.summarize_hamming_distances()
res = {}
for rnd in range(3):
    for name, chunk, keep in (("chunk262144", None, False), ("chunk131072", 131072, False), ("chunk65536", 65536, False),
                              ("chunk32768", 32768, False), ("keep_workspace", None, True)):
        _lib.keep_workspace(keep)
        with _lib.tuning(spectral_chunk=chunk):
            assert b.summarize_hamming_distances() == ref
            torch.cuda.synchronize()
            ts = []
            for _ in range(7):
                t = time.perf_counter()
                r = b.summarize_hamming_distances()
                ts.append((time.perf_counter() - t) * 1e3)
            assert r == ref
        _lib.keep_workspace(False)
        _lib.release_plan_cache()
        res.setdefault(name, []).append(sorted(ts)[3])
        print(json.dumps({"variant": name, "round": rnd, "median_ms": sorted(ts)[3]}), flush=True)
print(json.dumps({"summary": {k: min(v) for k, v in res.items()}}))
