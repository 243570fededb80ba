"""Host emulation of the SWAR byte tricks the encoders use instead of a byte LUT, checked
against the reference's maps (TwoBit encodings.py:53-69, ThreeBit encodings.py:139-149) over
every 4-byte word of a small alphabet (bases in both cases, N, IUPAC, '\\n', '\\r', others) and
every partial length.  v_perm_b32 is emulated byte for byte (selector 0-3: bytes of the second
source, 4-7: bytes of the first, 12: 0x00).  The kernels' own outputs are pinned on the GPU
(tests/test_gpu_parity.py); this pins the formulas themselves, on CPU."""
import itertools

import numpy as np

ALPHA = b"ACGTacgtNRY\n\rX"
TWO = {ord("A"): 0, ord("C"): 1, ord("T"): 2, ord("G"): 3}
THREE = {ord("C"): 1, ord("A"): 2, ord("G"): 3, ord("T"): 4}


def perm(s0, s1, sel):
    out = 0
    for i in range(4):
        k = (sel >> (8 * i)) & 0xFF
        if k < 4:
            v = (s1 >> (8 * k)) & 0xFF
        elif k < 8:
            v = (s0 >> (8 * (k - 4))) & 0xFF
        elif k == 12:
            v = 0
        else:
            v = 0xFF
        out |= v << (8 * i)
    return out


def words():
    for t in itertools.product(ALPHA, repeat=4):
        yield t, t[0] | t[1] << 8 | t[2] << 16 | t[3] << 24


def test_line_swar_twobit_threebit():
    """lines.hip encode_line1: upper-case A/C/G/T detected exactly; values packed MSB-first."""
    for kind in (2, 3):
        ref = TWO if kind == 2 else THREE
        for t, w in words():
            x = ((w >> 1) ^ (w >> 2)) & 0x03030303
            v = x ^ ((x >> 1) & 0x01010101)
            y = perm(0, v if kind == 2 else perm(0, 0x03040102, v), 0x00010203)
            if kind == 2:
                a = (y | (y >> 6)) & 0x000F000F
                pk = (a | (a >> 12)) & 0xFF
            else:
                a = (y | (y >> 5)) & 0x003F003F
                pk = (a | (a >> 10)) & 0xFFF
            for r in range(1, 5):
                keep = 0xFFFFFFFF if r == 4 else (1 << (8 * r)) - 1
                bad = (perm(0, 0x47544341, v) ^ w) & keep
                ok = all(c in b"ACGT" for c in t[:r])
                assert (bad == 0) == ok, (t, r)
                if ok:
                    want = 0
                    for c in t[:r]:
                        want = (want << kind) | ref[c]
                    assert pk >> (kind * (4 - r)) == want, (kind, t, r)


def test_tiled_encoder_masked_swar():
    """encode.hip encode_tiled_kernel (TwoBit): bases of either case packed by one multiply,
    every other byte's value cleared through the mismatch byte mask (its LUT code bits are 0),
    and exactly those bytes flagged for the LUT."""
    for t, w in words():
        u = w & 0xDFDFDFDF
        d = u ^ perm(0x47010154, 0x43014101, u & 0x07070707)
        nz = ((((d & 0x7F7F7F7F) + 0x7F7F7F7F) & 0xFFFFFFFF) | d) & 0x80808080
        bm = ((nz - (nz >> 7)) | nz) & 0xFFFFFFFF
        v = ((u >> 1) & 0x03030303) & ~bm & 0xFFFFFFFF
        code = ((v * 0x40100401) & 0xFFFFFFFF) >> 24
        want, flagged = 0, []
        for i, c in enumerate(t):
            cu = c & 0xDF
            if cu in TWO:
                want = (want << 2) | TWO[cu]
            else:
                want <<= 2  # lut & 7 == 0 for every non-base byte
                flagged.append(i)
        assert code == want, t
        assert [i for i in range(4) if (nz >> (8 * i + 7)) & 1] == flagged, t


def test_newline_count_bits():
    """fastq.hip fq_count_kernel / lines.hip lf_mask_v: bit 7 of each byte set iff it is '\\n'."""
    rng = np.random.default_rng(3)
    for _ in range(20000):
        b = rng.choice(list(ALPHA), 4)
        w = int(b[0]) | int(b[1]) << 8 | int(b[2]) << 16 | int(b[3]) << 24
        x = w ^ 0x0A0A0A0A
        hi = ~((((x & 0x7F7F7F7F) + 0x7F7F7F7F) & 0xFFFFFFFF) | x | 0x7F7F7F7F) & 0xFFFFFFFF
        assert bin(hi).count("1") == int((b == 10).sum())
        assert [i for i in range(4) if (hi >> (8 * i + 7)) & 1] == [i for i in range(4) if b[i] == 10]
        m4 = (((hi >> 7) * 0x10204080) & 0xFFFFFFFF) >> 28  # lines.hip lf_mask_v's gather
        assert m4 == sum(1 << i for i in range(4) if b[i] == 10)


def _lut(kind, c):
    """encode_common.h lut_entry: code in bits 0..2, 0x40 ambiguous / 0x80 invalid (TwoBit)."""
    u = chr(c).upper()
    if kind == 2:
        if u in "ACTG":
            return "ACTG".index(u)
        return 0x40 if u in "MRWSYKVHDBN" else 0x80
    return {"C": 1, "A": 2, "G": 3, "T": 4}.get(u, 6)


def _enc_bases(w, r, kind, code, fl):
    """fastq.hip enc_bases: r (1..4) bases of the dword w by SWAR, or -- when any of them is not an
    upper-case base -- its r bytes through the LUT, appended to code."""
    x = ((w >> 1) ^ (w >> 2)) & 0x03030303
    v = x ^ ((x >> 1) & 0x01010101)
    keep = 0xFFFFFFFF if r >= 4 else (1 << (8 * r)) - 1
    if (perm(0, 0x47544341, v) ^ w) & keep:
        for b in range(r):
            e = _lut(kind, (w >> (8 * b)) & 0xFF)
            code = (code << kind) | (e & 7)
            fl |= e
    else:
        if kind == 2:
            y = perm(0, v, 0x00010203)
            a = (y | (y >> 6)) & 0x000F000F
            pk = (a | (a >> 12)) & 0xFF
        else:
            y = perm(0, perm(0, 0x03040102, v), 0x00010203)
            a = (y | (y >> 5)) & 0x003F003F
            pk = (a | (a >> 10)) & 0xFFF
        code = (code << (kind * r)) | (pk >> (kind * (4 - r)))
    return code & ((1 << 64) - 1), fl


def test_fastq_window_encode():
    """fastq.hip line_spans: a slice of w <= 32 bytes encoded dword by dword from its 16-byte
    windows (enc_bases: SWAR, the LUT for a dword holding another byte) equals the per-byte LUT
    encode of the slice, flags included, for every width and mixes of bases, lower case, N, IUPAC
    and other bytes."""
    rng = np.random.default_rng(11)
    alpha = np.frombuffer(b"ACGTACGTACGTacgtNRY\nX", np.uint8)
    for kind, wmax in ((2, 32), (3, 21)):
        for w in range(1, wmax + 1):
            for trial in range(40):
                row = rng.choice(alpha[:4] if trial % 2 else alpha, w + 16).astype(np.uint8)
                code, fl = 0, 0
                for c in range(0, w, 16):
                    m = min(16, w - c)
                    for j in range(0, m, 4):
                        dw = int.from_bytes(bytes(row[c + j:c + j + 4]), "little")
                        code, fl = _enc_bases(dw, min(4, m - j), kind, code, fl)
                want, wfl = 0, 0
                for b in row[:w]:
                    e = _lut(kind, int(b))
                    want = (want << kind) | (e & 7)
                    wfl |= e
                assert code == want, (kind, w, bytes(row[:w]))
                assert fl & 0xC0 == wfl & 0xC0, (kind, w, bytes(row[:w]))  # the ambiguous / invalid flags
