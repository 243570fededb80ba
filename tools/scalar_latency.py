"""Per-call latency of the drop-in's scalar methods (batches of one through the C ABI and a
GPU round trip) against the reference's per-call times measured in the build container
(TwoBit.encode 2.7 us, hamming_distance 1.2 us, decode 2.1 us, gc_content
1.3 us; ThreeBit.encode 2.2 us, hamming 1.2 us).  Prints one JSON object."""

import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from sctools_amd import _lib, encodings  # noqa: E402

REF_US = {"TwoBit.encode": 2.7, "TwoBit.hamming_distance": 1.2, "TwoBit.decode": 2.1, "TwoBit.gc_content": 1.3,
          "ThreeBit.encode": 2.2, "ThreeBit.hamming_distance": 1.2}


def per_call_us(fn, args, reps):
    for a in args[:20]:
        fn(*a)
    t = time.perf_counter()
    for k in range(reps):
        fn(*args[k % len(args)])
    return (time.perf_counter() - t) / reps * 1e6


def main():
    _lib.check(_lib.lib().sct_set_device(0))
    rng = np.random.default_rng(1)
    seqs = [bytes(rng.choice(list(b"ACGT"), 16).tolist()) for _ in range(256)]
    T2, T3 = encodings.TwoBit, encodings.ThreeBit
    codes = [T2.encode(s) for s in seqs]
    c3 = [T3.encode(s) for s in seqs]
    t2 = T2(16)
    reps = int(os.environ.get("REPS", "2000"))
    out = {}
    out["TwoBit.encode"] = per_call_us(T2.encode, [(s,) for s in seqs], reps)
    out["TwoBit.hamming_distance"] = per_call_us(T2.hamming_distance, list(zip(codes, codes[1:])), reps)
    out["TwoBit.decode"] = per_call_us(t2.decode, [(c,) for c in codes], reps)
    out["TwoBit.gc_content"] = per_call_us(t2.gc_content, [(c,) for c in codes], reps)
    out["ThreeBit.encode"] = per_call_us(T3.encode, [(s,) for s in seqs], reps)
    out["ThreeBit.hamming_distance"] = per_call_us(T3.hamming_distance, list(zip(c3, c3[1:])), reps)
    # the raw C-ABI floor: one zero-copy hamming call of one pair, no Python wrapping
    a = np.array([codes[0]], dtype=np.uint64)
    b = np.array([codes[1]], dtype=np.uint64)
    o = np.zeros(1, dtype=np.int32)
    f = _lib.lib().sct_hamming_pairs_host
    pa, pb, po = a.ctypes.data, b.ctypes.data, o.ctypes.data
    out["c_abi.sct_hamming_pairs_host(n=1)"] = per_call_us(lambda: f(2, pa, pb, 1, 1, po), [()], reps)
    # batch throughput for scale
    big = np.array(codes * 4096, dtype=np.uint64)
    t = time.perf_counter()
    T2.hamming_distance_array(big, big[::-1].copy())
    out["TwoBit.hamming_distance_array(1M) us per pair"] = (time.perf_counter() - t) / big.size * 1e6
    print(json.dumps({"unit": "us per call", "measured": out, "reference_us": REF_US}))


if __name__ == "__main__":
    main()
