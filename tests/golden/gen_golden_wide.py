"""Golden fixtures for all-pairs summaries over keys >= 2^64, generated from the REFERENCE.

Barcodes.summarize_hamming_distances (src/sctools/barcode.py:39-46) takes Python ints of any
size: ThreeBit-encoded 22..28-bp barcodes (66..84 bits), TwoBit-encoded barcodes longer than
32 bp, and sets that mix narrow and wide keys.  This script imports the reference through
the loader shim of gen_golden.py (build container only) and writes inputs plus the
reference's own summary and distance histogram to tests/golden/wide_sets.json.

Usage:  python tests/golden/gen_golden_wide.py
"""

import itertools
import json
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from gen_golden import load_reference, summary_record  # noqa: E402


def main():
    enc, bc, _ = load_reference()
    TwoBit, ThreeBit = enc.TwoBit, enc.ThreeBit
    rng = random.Random(20261016)
    sets = []

    def add(kind, L, seqs, codes):
        bset = bc.Barcodes.from_iterable_encoded(codes, barcode_length=L)
        keys = list(bset)
        hist = np.bincount([TwoBit.hamming_distance(a, b) for a, b in itertools.combinations(keys, 2)],
                           minlength=1).tolist()
        rec = {"kind": kind, "L": L, "codes": [str(c) for c in codes], "hist": hist}
        try:
            rec["summary"] = summary_record(bset.summarize_hamming_distances())
        except IndexError as e:
            rec["error"] = {"type": "IndexError", "args": list(e.args)}
        if seqs is not None:
            rec["seqs"] = [s.hex() for s in seqs]
        sets.append(rec)

    # ThreeBit-encoded 22..28-bp whitelists (the keys summarize with the TwoBit distance)
    for L in range(22, 29):
        for n in (2, 3, 60, 400):
            seqs = [bytes(rng.choice(b"ACGTN" if rng.random() < 0.1 else b"ACGT") for _ in range(L)) for _ in range(n)]
            add("three", L, seqs, [ThreeBit.encode(s) for s in seqs])
    # one larger set at the 10x v3-length bound
    seqs = [bytes(rng.choice(b"ACGT") for _ in range(28)) for _ in range(1500)]
    seqs += [s[:5] + b"N" + s[6:] for s in seqs[:40]]  # near neighbours
    add("three", 28, seqs, [ThreeBit.encode(s) for s in seqs])
    # TwoBit keys longer than 32 bp, and sets mixing narrow and wide keys
    for L in (33, 40, 64, 65, 100):
        seqs = [bytes(rng.choice(b"ACGT") for _ in range(L)) for _ in range(150)]
        add("two", L, seqs, [TwoBit.encode(s) for s in seqs])
    for _ in range(6):
        codes = [rng.getrandbits(rng.choice((16, 32, 63, 64, 65, 84, 130, 200, 300))) for _ in range(rng.randint(2, 80))]
        codes += codes[:3]  # duplicates collapse in Counter
        add("mixed", 16, None, codes)

    with open(os.path.join(HERE, "wide_sets.json"), "w") as f:
        json.dump(sets, f, separators=(",", ":"))
    print("wrote wide_sets.json: %d sets" % len(sets))


if __name__ == "__main__":
    main()
