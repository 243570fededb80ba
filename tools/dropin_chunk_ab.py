"""The drop-in call at several SPECTRAL chunk sizes, both memory policies: each chunk of 2^k slices
needs a 2^(k+14)-byte intermediate (the default policy maps and unmaps it per call; keep_workspace
caches it), so a smaller chunk maps less but launches the seed / tile pair more often; at 2^13
slices (128 MiB) the intermediate fits the 256-MB Infinity Cache.  Barcodes(dict of config 2).
summarize_hamming_distances(), wall-clock medians of 7, rounds interleaved."""
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
# (None: the library's default -- 65536 slices for the one-shot call since round 6, 262144 cached)
variants = [("default_chunk%s" % (c or "65536"), c, False) for c in (None, 262144, 32768)] + \
           [("keep_chunk%s" % (c or "262144"), c, True) for c in (None,)]
for rnd in range(4):
    for name, chunk, keep in variants:
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
print(json.dumps({"summary": {k: sorted(v)[len(v) // 2] for k, v in res.items()}}))
