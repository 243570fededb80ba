"""Seeded synthetic barcode sets for the benchmark configs.

Host-side data generation only (no reference code, no GPU). Every 2L-bit
unsigned integer is a valid TwoBit code of an L-bp barcode
(``encodings.py:63-69`` maps each base to 2 bits), so a whitelist is drawn
directly as uniformly random codes, de-duplicated the way ``Barcodes``
de-duplicates through ``collections.Counter`` (``barcode.py:97``), and topped
up until it holds exactly ``n`` unique codes.
"""

import numpy as np

#: BASELINE.json configs -> (n, L, seed) of the whitelist (config 3 = config 2's set over 2/4/8
#: GPUs; config 4's whitelist is config 2's set, ThreeBit-encoded, queried by CONFIG4_QUERIES
#: observed barcodes; config 5 also streams CONFIG5_READS 28-bp reads)
CONFIGS = {
    1: (10_000, 16, 1),
    2: (737_280, 16, 737_280),
    3: (737_280, 16, 737_280),
    4: (737_280, 16, 737_280),
    5: (3_686_400, 16, 5),
}
CONFIG4_QUERIES = 100_000_000
CONFIG5_READS, CONFIG5_READ_LENGTH = 1_000_000_000, 28


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


def two_to_three(codes2, barcode_length=16):
    """TwoBit codes -> ThreeBit codes of the same sequence (A0 C1 T2 G3 -> A2 C1 T4 G3;
    encodings.py:58-59 vs :142-143)."""
    m = np.array([2, 1, 4, 3], dtype=np.uint64)
    codes2 = np.asarray(codes2, dtype=np.uint64)
    out = np.zeros(codes2.size, dtype=np.uint64)
    for p in range(barcode_length):
        v = (codes2 >> np.uint64(2 * p)) & np.uint64(3)
        out |= m[v.astype(np.intp)] << np.uint64(3 * p)
    return out


def config4_queries(wl3, nq, seed=4, barcode_length=16, device=None):
    """Config 4's observed barcodes as ThreeBit codes, built on `device` (a torch device):
    50 % exact whitelist draws, 25 % one substitution (A/C/G/T), 15 % one N, 10 % uniformly
    random ACGT.  Returns (queries int64 tensor, picked whitelist index, class tensor: 0
    exact, 1 substitution, 2 N, 3 random)."""
    import torch
    L = barcode_length
    dev = device or torch.device("cuda")
    d_wl = torch.as_tensor(np.ascontiguousarray(wl3, dtype=np.uint64).view(np.int64), device=dev)
    g = torch.Generator(device=dev).manual_seed(seed)
    n = d_wl.numel()
    pick = torch.randint(0, n, (nq,), device=dev, generator=g)
    q = d_wl[pick].clone()
    u = torch.rand(nq, device=dev, generator=g)
    pos = torch.randint(0, L, (nq,), device=dev, generator=g) * 3
    base = torch.randint(1, 5, (nq,), device=dev, generator=g)
    clear = ~(torch.full_like(q, 7) << pos)
    sub = (u >= 0.5) & (u < 0.75)
    q = torch.where(sub, (q & clear) | (base << pos), q)
    nmask = (u >= 0.75) & (u < 0.9)
    q = torch.where(nmask, (q & clear) | (torch.full_like(q, 6) << pos), q)
    rnd = u >= 0.9
    r = torch.zeros_like(q)
    for p in range(L):
        r |= torch.randint(1, 5, (nq,), device=dev, generator=g) << (3 * p)
    q = torch.where(rnd, r, q)
    cls = sub.to(torch.int8) + 2 * nmask.to(torch.int8) + 3 * rnd.to(torch.int8)
    return q, pick, cls
