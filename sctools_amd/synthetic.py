"""Seeded synthetic barcode sets for the benchmark configs.

Host-side data generation only (no reference code, no GPU). Every 2L-bit
unsigned integer is a valid TwoBit code of an L-bp barcode
(``encodings.py:63-69`` maps each base to 2 bits), so a whitelist is drawn
directly as uniformly random codes, de-duplicated the way ``Barcodes``
de-duplicates through ``collections.Counter`` (``barcode.py:97``), and topped
up until it holds exactly ``n`` unique codes.
"""

import numpy as np

#: BASELINE.json configs -> (n, L, seed)
CONFIGS = {
    1: (10_000, 16, 1),
    2: (737_280, 16, 737_280),
    5: (3_686_400, 16, 5),
}


def whitelist_codes(n, barcode_length=16, seed=1):
    """Return ``n`` unique TwoBit codes (np.uint64, sorted ascending)."""
    if barcode_length < 1 or barcode_length > 32:
        raise ValueError("barcode_length must be in [1, 32]")
    space = 4 ** barcode_length
    if n > space:
        raise ValueError("cannot draw %d unique %d-bp barcodes" % (n, barcode_length))
    rng = np.random.default_rng(seed)

    def draw(k):
        if barcode_length == 32:
            return rng.integers(0, 2 ** 64, size=k, dtype=np.uint64, endpoint=False)
        return rng.integers(0, space, size=k, dtype=np.uint64)

    codes = np.unique(draw(n))
    while codes.size < n:
        codes = np.unique(np.concatenate([codes, draw(n - codes.size)]))
    return codes


def decode_ascii(codes, barcode_length):
    """TwoBit codes -> (n, L) uint8 ASCII array (MSB-first, ``encodings.py:90-100``)."""
    codes = np.asarray(codes, dtype=np.uint64)
    lut = np.frombuffer(b"ACTG", dtype=np.uint8)
    shifts = np.arange(barcode_length - 1, -1, -1, dtype=np.uint64) * np.uint64(2)
    idx = (codes[:, None] >> shifts[None, :]) & np.uint64(3)
    return lut[idx.astype(np.intp)]
