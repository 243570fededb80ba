"""Host emulation of the tile-prefix scheme (sctools_amd/csrc/tile_prefix.h) the ingest kernels
number their lines with: per-tile counts / last positions (c0 / l0), the one-wave reduction into
blocks of 32 and 1,024 tiles (tile_sums_reduce_kernel), and a tile's exclusive prefix from at
most (t >> 10) + 31 + 31 of those values (tile_prefix) -- against a plain cumulative sum, for
tile counts around the block edges.  The GPU parity tests pin the kernels; this pins the index
arithmetic on CPU."""
import numpy as np
import pytest


def reduce_levels(c0, l0):
    n = c0.size
    n1, n2 = (n + 31) >> 5, (n + 1023) >> 10
    c1 = np.zeros(n1, np.int64)
    l1 = np.zeros(n1, np.int64)
    c2 = np.zeros(n2, np.int64)
    l2 = np.zeros(n2, np.int64)
    for b in range(n2):  # one wave per 1,024 tiles: lane i sums tiles [16 i, 16 i + 16)
        for lane in range(64):
            t0 = b * 1024 + 16 * lane
            seg = slice(t0, min(t0 + 16, n))
            if t0 >= n:
                continue
            c, l = int(c0[seg].sum()), int(l0[seg].max(initial=0))
            c2[b] += c
            l2[b] = max(l2[b], l)
            c1[t0 >> 5] += c  # lane pairs form the 32-tile sums
            l1[t0 >> 5] = max(l1[t0 >> 5], l)
    return c1, l1, c2, l2


def prefix(t, c0, l0, c1, l1, c2, l2):
    A, B, C = t >> 10, (t >> 5) & 31, t & 31
    s, m = 0, 0
    for j in range(A + B + C):
        if j < A:
            k, cp, lq = j, c2, l2
        elif j < A + B:
            k, cp, lq = (t >> 10) * 32 + (j - A), c1, l1
        else:
            k, cp, lq = (t >> 5) * 32 + (j - A - B), c0, l0
        s += int(cp[k])
        m = max(m, int(lq[k]))
    return s, m - 1


@pytest.mark.parametrize("ntiles", [1, 31, 32, 33, 1023, 1024, 1025, 2080, 3826])
def test_tile_prefix_matches_cumsum(ntiles):
    rng = np.random.default_rng(ntiles)
    c0 = rng.integers(0, 300, ntiles).astype(np.int64)
    c0[rng.random(ntiles) < 0.2] = 0  # tiles with no line end
    # last position + 1 of each tile (0: none): increasing with the tile, as in a buffer
    l0 = np.where(c0 > 0, np.arange(ntiles) * 16384 + rng.integers(1, 16385, ntiles), 0).astype(np.int64)
    c1, l1, c2, l2 = reduce_levels(c0, l0)
    want_c = np.concatenate([[0], np.cumsum(c0)[:-1]])
    want_l = np.concatenate([[0], np.maximum.accumulate(l0)[:-1]]) - 1
    for t in sorted({0, 1, 31, 32, 33, 1023, 1024, 1025, ntiles - 1} & set(range(ntiles))):
        assert prefix(t, c0, l0, c1, l1, c2, l2) == (int(want_c[t]), int(want_l[t])), t
