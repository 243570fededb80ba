"""Generate tests/golden/edges.json: the drop-in's API-boundary edge cases, from the
REFERENCE itself (VERDICT r4 "What's weak" #1).

Same loader shim as gen_golden.py (a stub ``sctools`` package so ``__init__.py`` never
runs, plus the ``collections.Mapping`` alias). Only calls the reference makes finish
on are recorded; the calls on which its digit loops never end (a negative XOR in
``hamming_distance``, encodings.py:117-120; a negative value in ThreeBit
``gc_content``, encodings.py:189) are listed under ``hangs`` with no expected value:
the drop-in raises ValueError there instead.

Usage:  python tests/golden/gen_golden_edges.py
"""

import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from gen_golden import exc_record, load_reference  # noqa: E402


def call(fn, *args):
    try:
        r = fn(*args)
    except Exception as e:  # the reference's own exception, recorded by type and args
        return {"error": exc_record(e)}
    if isinstance(r, bytes):
        return {"bytes": r.hex()}
    return {"value": str(r)}


def iterable_from_spec(spec):
    """The items of an edges.json from_iterable_strings case, as a generator (tests rebuild
    them with the same function: tests/test_gpu_parity.py imports it from here)."""
    for item in spec:
        tag = item[0]
        if tag == "raise":
            raise RuntimeError(item[1])
        yield {"s": lambda v: v, "b": bytes.fromhex, "i": int, "f": float, "n": lambda *a: None}[tag](*item[1:])


def main():
    enc, bc, _ = load_reference()
    TwoBit, ThreeBit = enc.TwoBit, enc.ThreeBit
    rng = random.Random(20261018)
    out = {}

    # ---- TwoBit decode / gc_content of negative ints (encodings.py:90-111): the loop
    # runs sequence_length times, so the value is read mod 4**L
    neg2 = []
    fixed = [-1, -2, -3, -4, -5, -16, -(2 ** 31), -(2 ** 32), -(2 ** 63), -(2 ** 64), -(2 ** 64) - 1,
             -(2 ** 70), -(2 ** 70) + 12345, -(2 ** 128) - 7]
    for L in (0, 1, 2, 3, 4, 8, 16, 21, 31, 32, 33, 40, 64, 65, 70):
        vals = list(fixed) + [-rng.getrandbits(rng.choice((8, 32, 63, 64, 65, 100, 150))) - 1 for _ in range(12)]
        for x in vals:
            t = TwoBit(L)
            neg2.append({"L": L, "code": str(x), "decode": call(t.decode, x), "gc": call(t.gc_content, x)})
    out["twobit_negative"] = neg2

    # ---- hamming_distance of two negatives (encodings.py:113-121, 194-202): a ^ b >= 0
    ham = []
    pairs = [(-1, -2), (-(2 ** 70), -3), (-1, -1), (-5, -(2 ** 64)), (-(2 ** 63), -1), (-(2 ** 64), -(2 ** 64) - 1),
             (-(2 ** 200), -(2 ** 199)), (-7, -8), (-(2 ** 65) + 3, -(2 ** 20))]
    for _ in range(400):
        ba, bb = rng.choice((4, 16, 32, 62, 63, 64, 65, 84, 128, 190)), rng.choice((4, 32, 63, 64, 65, 128))
        a = -rng.getrandbits(ba) - 1
        b = a ^ (rng.getrandbits(5) << rng.randrange(ba)) if rng.random() < 0.4 else -rng.getrandbits(bb) - 1
        if b >= 0:
            b = ~b
        pairs.append((a, b))
    for a, b in pairs:
        ham.append([str(a), str(b), TwoBit.hamming_distance(a, b), ThreeBit.hamming_distance(a, b)])
    out["hamming_negative"] = ham

    # ---- ThreeBit.decode of negative ints (encodings.py:169-180): the value converges to
    # -1, whose triplet 7 is not in the decoding map, so every negative input raises
    # KeyError at its lowest 0/5/7 triplet
    dec3 = []
    for x in [-1, -2, -6, -7, -8, -9, -0o12, -0o1234, -(2 ** 63), -(2 ** 64), -(2 ** 66) + 0o1234]:
        dec3.append({"code": str(x), "decode": call(ThreeBit.decode, x)})
    for _ in range(60):
        # lows of valid triplets above an all-ones (negative) top
        k = rng.randint(1, 30)
        low = 0
        for _ in range(k):
            low = (low << 3) | rng.choice((1, 2, 3, 4, 6))
        x = low - (1 << (3 * k))  # low triplets valid, then the sign extension (7s)
        if rng.random() < 0.3:
            x ^= rng.choice((0, 5, 7)) << (3 * rng.randrange(k))
            if x >= 0:
                x = ~x
        dec3.append({"code": str(x), "decode": call(ThreeBit.decode, x)})
    out["threebit_decode_negative"] = dec3

    # ---- Barcodes.from_iterable_bytes on non-bytes items (barcode.py:111-114)
    ib = []
    for name, items, L in (
            ("ints", [5, 6], 4),
            ("int_after_bytes", [b"ACGT", 7], 4),
            ("str", ["ACGT"], 4),
            ("empty_str", [""], 4),
            ("list_of_ints", [[65, 67, 71, 84], [84, 84, 65, 65]], 4),
            ("bytearray", [bytearray(b"ACGT"), memoryview(b"TTGA")], 4),
            ("tuple_of_ints", [(65, 67)], 2),
            ("none", [None], 4),
            ("float", [1.5], 4)):
        rec = {"name": name, "L": L}
        try:
            s = bc.Barcodes.from_iterable_bytes(items, L)
            rec["codes"] = [str(k) for k in s]
            rec["counts"] = [s[k] for k in s]
        except Exception as e:
            rec["error"] = exc_record(e)
        ib.append(rec)
    out["from_iterable_bytes"] = ib

    # ---- Barcodes.from_iterable_strings (barcode.py:104-108): `b.encode()` and the encode run
    # item by item inside the Counter's generator, so an item that fails raises only after the
    # items before it made their random draws, and an earlier item's KeyError comes first.
    # Items are JSON specs (built by iterable_from_spec): ["s", str], ["b", hex bytes],
    # ["i", int], ["f", float], ["n"] (None), ["raise", msg] (the iterable raises RuntimeError)
    fs = []
    for name, spec, L, seed in (
            ("keyerror_before_attr", [["s", "ACGP"], ["i", 5]], 4, 11),
            ("draws_before_attr", [["s", "ANNA"], ["i", 5]], 4, 12),
            ("none", [["n"]], 4, 13),
            ("bytes_item", [["s", "ACGT"], ["b", "41434754"]], 4, 14),
            ("float_after_n", [["s", "NNNN"], ["f", 1.5]], 4, 15),
            ("non_ascii", [["s", "NN"], ["s", "ACéG"], ["s", "NNNN"]], 4, 16),
            ("keyerror_mid", [["s", "NNNN"], ["s", "ACGX"], ["s", "NNNN"]], 4, 17),
            ("generator_raises", [["s", "ACGT"], ["s", "NNAC"], ["raise", "boom"], ["s", "NNNN"]], 4, 18),
            ("raises_after_bad", [["s", "NACGTX"], ["raise", "boom"]], 6, 19),
            ("ok_ragged", [["s", "ACGT"], ["s", "NN"], ["s", "ACGTNA"], ["s", "ACGT"], ["s", ""]], 4, 20),
            ("ok_with_n", [["s", "ANNA"], ["s", "acgt"], ["s", "ANNA"], ["s", "ryky"]], 4, 21),
            ("empty", [], 4, 22)):
        rec = {"name": name, "spec": spec, "L": L, "seed": seed}
        random.seed(seed)
        try:
            s = bc.Barcodes.from_iterable_strings(iterable_from_spec(spec), L)
            rec["codes"] = [str(k) for k in s]
            rec["counts"] = [s[k] for k in s]
        except Exception as e:
            rec["error"] = exc_record(e)
        rec["after"] = random.getrandbits(32)
        fs.append(rec)
    out["from_iterable_strings"] = fs

    # calls the reference never returns from (not executed here)
    out["hangs"] = {
        "hamming_mixed_signs": [["-1", "0"], ["-1", "1"], ["5", "-3"], [str(-(2 ** 70)), "1"]],
        "threebit_gc_negative": ["-1", "-8", str(-(2 ** 70))],
    }

    with open(os.path.join(HERE, "edges.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print("wrote edges.json")


if __name__ == "__main__":
    main()
