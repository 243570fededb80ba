"""Host-only check of the seed kernels' walk bookkeeping (sctools_amd/csrc/spectral.hip
seed_walks / walk_from, spectral16.hip seed16_walks), restated in
Python: every 64-slice walk runs from the XOR of the planes of its slice bits 6 and up, its
last state is that start with plane 5 flipped, and the Gray-ordered blocks of 2^lp walks
reach every walk of a range exactly once with the state the direct computation gives."""
import random

import pytest


def start_state(planes, zblk, walk_bits=6):
    x = 0
    for k in range(walk_bits, len(planes)):
        if (zblk >> k) & 1:
            x ^= planes[k]
    return x


def walk(planes, x):
    """the 64 Gray steps of walk_from: returns (states visited, the last state)"""
    seen = [x]
    for i in range(1, 64):
        x ^= planes[(i & -i).bit_length() - 1]
        seen.append(x)
    return seen, x


@pytest.mark.parametrize("nplanes", [18, 16])
def test_walk_ends_with_plane5_flipped(nplanes):
    rng = random.Random(nplanes)
    planes = [rng.getrandbits(32) for _ in range(nplanes)]
    for zblk in (0, 64, 64 * 37, (1 << nplanes) - 64):
        x0 = start_state(planes, zblk)
        seen, last = walk(planes, x0)
        assert last == x0 ^ planes[5]
        # step i visits slice zblk + gray(i): its state is the direct XOR of that slice's planes
        for i, x in enumerate(seen):
            z = zblk + (i ^ (i >> 1))
            assert x == start_state(planes, z, walk_bits=0)


@pytest.mark.parametrize("lp", [0, 1, 3, 4])
def test_gray_blocks_cover_the_range_with_direct_states(lp):
    rng = random.Random(lp)
    planes = [rng.getrandbits(32) for _ in range(18)]
    for z0, z1 in ((0, 1 << 18), (64 * 5 + 7, 64 * 300 + 1), (64 * 1000, 64 * 1000 + 64), (33, 40)):
        wa, we, P = (z0 & ~63) >> 6, (z1 + 63) >> 6, 1 << lp
        visited = []
        for b in range(wa >> lp, (we + P - 1) >> lp):  # every workgroup row, in any order
            x = start_state(planes, (b << lp) << 6)
            for j in range(P):
                if j:
                    t = (j & -j).bit_length() - 1
                    x ^= planes[5] ^ planes[6 + t]
                w = (b << lp) + (j ^ (j >> 1))
                if w < wa or w >= we:
                    x ^= planes[5]
                    continue
                assert x == start_state(planes, w << 6), (z0, z1, lp, b, j)
                visited.append(w)
                _, x = walk(planes, x)
        assert sorted(visited) == list(range(wa, we))
