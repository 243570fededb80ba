"""GPU: the resident scalar server behind the drop-in's scalar calls (encode.hip,
`scalar_server_kernel`).  Calls of <= 64 records are answered by a one-wave kernel that
polls a host-coherent mailbox; these tests check its answers against the oracle (the
reference's own per-call semantics, encodings.py:75-202) and its life cycle: first-call
launch, idle exit and relaunch, explicit stop, the stop before persistent-grid kernels,
and one server per host thread."""
import ctypes
import random
import threading
import time

import numpy as np
import pytest

from oracle import oracle as O
from sctools_amd import _lib, barcode, encodings

pytestmark = pytest.mark.gpu

T2, T3 = encodings.TwoBit, encodings.ThreeBit


def status():
    launches, running = ctypes.c_int64(), ctypes.c_int32()
    _lib.check(_lib.lib().sct_scalar_server_status(ctypes.byref(launches), ctypes.byref(running)))
    return launches.value, running.value


def _rand_seq(rng, L, alphabet=b"ACGT"):
    return bytes(rng.choice(list(alphabet), L).tolist())


def test_scalar_calls_use_the_server_and_match_the_oracle():
    rng = np.random.default_rng(5)
    _lib.check(_lib.lib().sct_set_device(0))
    before, _ = status()
    for _ in range(300):
        L = int(rng.integers(1, 33))
        s = _rand_seq(rng, L)
        c = T2.encode(s)
        assert c == O.two_bit_encode(s)
        t = T2(L)
        assert t.decode(c) == O.two_bit_decode(c, L)
        assert t.gc_content(c) == O.two_bit_gc(c, L)
        d = random.Random(L * 7919 + len(s)).getrandbits(2 * L)
        assert T2.hamming_distance(c, d) == O.two_bit_hamming(c, d)
        L3 = int(rng.integers(1, 22))
        s3 = _rand_seq(rng, L3, b"ACGTN")
        c3 = T3.encode(s3)
        assert c3 == O.three_bit_encode(s3)
        assert T3.decode(c3) == O.three_bit_decode(c3)
        assert T3.gc_content(c3) == O.three_bit_gc(c3)
        e3 = T3.encode(_rand_seq(rng, L3, b"ACGTN"))
        assert T3.hamming_distance(c3, e3) == O.three_bit_hamming(c3, e3)
    after, running = status()
    assert after >= before + 1 and running >= 1
    # a tight loop keeps one server alive: far fewer launches than calls
    assert after - before < 50


def test_small_batches_up_to_64_records():
    rng = np.random.default_rng(6)
    for n in (1, 2, 17, 63, 64, 65):
        seqs = [_rand_seq(rng, 16) for _ in range(n)]
        codes, gc = T2.encode_array(seqs, return_gc=True)
        want = [O.two_bit_encode(s) for s in seqs]
        assert [int(x) for x in codes] == want
        assert [int(g) for g in gc] == [O.two_bit_gc(c, 16) for c in want]
        other = np.array([O.two_bit_encode(_rand_seq(rng, 16)) for _ in range(n)], dtype=np.uint64)
        got = T2.hamming_distance_array(np.asarray(want, dtype=np.uint64), other)
        assert [int(d) for d in got] == [O.two_bit_hamming(a, int(b)) for a, b in zip(want, other)]
        dec = T2(16).decode_array(np.asarray(want, dtype=np.uint64))
        assert [bytes(x) for x in dec] == [O.two_bit_decode(c, 16) for c in want]


def test_multi_limb_and_invalid_records_through_the_server():
    """Two-limb TwoBit codes (L 33-40) and ThreeBit decode errors (KeyError 0/5/7) keep the
    reference's semantics on the server path."""
    rng = np.random.default_rng(7)
    for L in (33, 40):
        s = _rand_seq(rng, L)
        c = T2.encode(s)
        assert c == O.two_bit_encode(s)
        assert T2(L).decode(c) == O.two_bit_decode(c, L)
    for bad in (0b101, 0b111, (0b001 << 3) | 0b101):
        with pytest.raises(KeyError):
            T3.decode(bad)
    random.seed(3)
    want = O.two_bit_encode(b"ACNNGT")
    random.seed(3)
    assert T2.encode(b"ACNNGT") == want
    with pytest.raises(KeyError):
        T2.encode(b"ACXT")


def test_idle_exit_relaunch_and_stop():
    lib = _lib.lib()
    assert T2.hamming_distance(5, 6) == O.two_bit_hamming(5, 6)
    l0, r0 = status()
    assert r0 >= 1
    time.sleep(0.2)  # > the 5 ms idle limit
    l1, r1 = status()
    assert r1 == 0 and l1 == l0
    assert T2.hamming_distance(7, 1) == O.two_bit_hamming(7, 1)
    l2, r2 = status()
    assert l2 == l1 + 1 and r2 >= 1
    _lib.check(lib.sct_scalar_server_stop())
    assert status()[1] == 0
    assert T2(4).gc_content(0b11011101) == O.two_bit_gc(0b11011101, 4)


def test_persistent_grid_kernels_stop_the_server_first():
    rng = np.random.default_rng(8)
    codes = sorted({int(x) for x in rng.integers(0, 4 ** 16, 3000)})
    T2.hamming_distance(codes[0], codes[1])
    assert status()[1] >= 1
    s = barcode.Barcodes({c: 1 for c in codes}, 16)
    got = s.summarize_hamming_distances()
    assert status()[1] == 0
    assert got == O.summary_from_hist_numpy(O.allpairs_hist_numpy(codes))


def test_one_server_per_thread():
    errors = []

    def work(seed):
        rng = np.random.default_rng(seed)
        _lib.check(_lib.lib().sct_set_device(0))
        try:
            for _ in range(200):
                a, b = (int(x) for x in rng.integers(0, 4 ** 16, 2))
                if T2.hamming_distance(a, b) != O.two_bit_hamming(a, b):
                    errors.append((a, b))
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    ts = [threading.Thread(target=work, args=(k,)) for k in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=60)
    assert not errors
    assert not any(t.is_alive() for t in ts)


def test_cpython_entry_points_take_the_common_case():
    """The scalar methods' C entry points (csrc/pyscalar.c) answer ints in [0, 2^64) and one-limb
    bytes records themselves, equal to the ctypes path, and leave every other case (negative or
    multi-limb ints, numpy scalars, str, ambiguous bases, L = 0 or > 64) to the Python path."""
    from sctools_amd import _scalar
    _lib.lib()  # binds the entry points
    rng = random.Random(17)
    for kind in (2, 3):
        for _ in range(200):
            a, b = rng.getrandbits(64), rng.getrandbits(rng.choice((1, 20, 63, 64)))
            assert _scalar.hamming(kind, a, b) == _lib.hamming1(kind, a, b)
            assert _scalar.gc(kind, a, 32 if kind == 2 else 0) == _lib.gc1(kind, a, 32 if kind == 2 else 0)
        for L in (1, 7, 16, 21):
            s = bytes(rng.choice(b"ACGT") for _ in range(L))
            assert _scalar.encode(kind, s) == _lib.encode1(kind, s)[0]
    for L in (1, 16, 33, 64):
        x = rng.getrandbits(2 * L) & ((1 << 64) - 1)
        assert _scalar.decode2(x, L) == _lib.decode2_1(x, L)
    assert _scalar.hamming(2, True, False) == 1
    for args in ((2, -1, 3), (2, 1 << 64, 3), (2, np.uint64(3), 1), (2, 1.0, 1)):
        assert _scalar.hamming(*args) is NotImplemented
    assert _scalar.gc(2, 5, 0) is NotImplemented and _scalar.gc(2, -5, 8) is NotImplemented
    assert _scalar.decode2(5, 0) is NotImplemented and _scalar.decode2(5, 65) is NotImplemented
    assert _scalar.encode(2, b"ACNT") is NotImplemented  # ambiguous: drawn in order by the Python path
    assert _scalar.encode(3, b"ACNT") == _lib.encode1(3, b"ACNT")[0]  # ThreeBit keeps N
    for seq in ("ACGT", bytearray(b"ACGT"), b"", b"A" * 33):
        assert _scalar.encode(2, seq) is NotImplemented
    assert _scalar.encode(3, b"A" * 22) is NotImplemented
    for s in (b"A", b"ACGTN" * 4, b"T" * 21):
        c = T3.encode(s)
        assert _scalar.decode3(c) == s == T3.decode_array([c])[0]
    assert _scalar.decode3(0) == b"" and _scalar.decode3(5) is NotImplemented  # KeyError(5) via Python
    assert _scalar.decode3(-1) is NotImplemented and _scalar.decode3(1 << 64) is NotImplemented
