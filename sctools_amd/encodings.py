"""Drop-in for ``sctools.encodings`` (src/sctools/encodings.py) on MI355X.

Same classes, attributes and method signatures as the reference; every encode,
decode, gc_content and hamming_distance call runs as a HIP kernel through
``libsctools_hip.so`` (scalar methods are batches of one).  Batch methods
(``*_array``) take and return numpy arrays.

The only host-side step is the reference's own RNG contract: TwoBit draws
``random.randint(0, 3)`` from the GLOBAL ``random`` module for every IUPAC
ambiguity code, in record order and left to right (encodings.py:63-69).  The
kernel encodes such bases as 0 and flags the record; the flagged records are then
walked here, in order, drawing exactly the numbers the reference would draw (and
raising its KeyError at the first invalid byte, after the draws that precede it).
"""

import operator
import random

import numpy as np

from . import _lib, _scalar

__all__ = ["Encoding", "TwoBit", "ThreeBit"]

_AMBIGUOUS = frozenset(b"MRWSYKVHDBNmrwsykvhdbn")  # encodings.py:61
_VALID2 = {ord("A"): 0, ord("C"): 1, ord("T"): 2, ord("G"): 3,
           ord("a"): 0, ord("c"): 1, ord("t"): 2, ord("g"): 3}  # encodings.py:58-59


def _as_bytes(seq):
    """bytes-like -> bytes, mirroring what iterating the reference's input yields."""
    if isinstance(seq, (bytes, bytearray, memoryview)):
        return bytes(seq)
    if isinstance(seq, np.ndarray) and seq.dtype == np.uint8:
        return seq.tobytes()
    return bytes(seq)  # iterable of ints in [0, 255]


def _records(seqs):
    """Batch input -> (n, L) uint8 array of equal-length records."""
    if isinstance(seqs, np.ndarray):
        if seqs.dtype.kind == "S":  # (a view of the rows: no copy)
            L = seqs.dtype.itemsize
            return np.ascontiguousarray(seqs).reshape(-1).view(np.uint8).reshape(-1, L)
        if seqs.dtype == np.uint8 and seqs.ndim == 2:
            return np.ascontiguousarray(seqs)
        raise TypeError("expected an 'S<L>' array or an (n, L) uint8 array")
    seqs = [_as_bytes(s) for s in seqs]
    if not seqs:
        return np.zeros((0, 0), dtype=np.uint8)
    L = len(seqs[0])
    if any(len(s) != L for s in seqs):
        raise ValueError("encode_array needs equal-length records; use encode() per record")
    return np.frombuffer(b"".join(seqs), dtype=np.uint8).reshape(len(seqs), L)


_STREAM_MIN_RECORDS = 1 << 20
_U64 = 1 << 64


def _encode_records(kind, recs):
    """Large one-limb batches go through the pipelined H2D/encode/D2H stream."""
    n, L = recs.shape
    if n >= _STREAM_MIN_RECORDS and 1 <= L and kind * L <= 64:
        codes, gc, flags = _lib.encode_stream(kind, recs)
        return codes.reshape(n, 1), gc, flags
    return _lib.encode(kind, recs, L)


def _fill_ambiguous(recs, codes, gc, flags):
    """Walk flagged TwoBit records in order: draw random.randint(0,3) per ambiguous
    byte (encodings.py:69) and raise the reference's KeyError on an invalid one (:68)."""
    hot = np.flatnonzero(flags)
    if hot.size == 0:
        return
    L = recs.shape[1]
    words = codes.shape[1]
    for r in hot.tolist():
        rec = recs[r]
        add = 0
        for p in range(L):
            byte = int(rec[p])
            if byte in _VALID2:
                continue
            if byte not in _AMBIGUOUS:
                raise KeyError('%s is not a valid IUPAC nucleotide code' % chr(byte))
            v = random.randint(0, 3)
            add |= v << (2 * (L - 1 - p))
            if gc is not None:
                gc[r] += v & 1
        if add:
            if words == 1:
                codes[r, 0] |= np.uint64(add)
            else:
                full = _lib.limbs_to_ints(codes[r:r + 1])[0] | add
                codes[r] = _lib.ints_to_limbs([full], words)[0]


def _limbs_of(values):
    """ints / uint64 array -> (n, words) uint64 limbs (rejects negatives)."""
    if isinstance(values, np.ndarray) and values.dtype.kind in "ui":
        if values.dtype.kind == "i" and values.size and values.min() < 0:
            raise ValueError("encoded values must be non-negative")
        return np.ascontiguousarray(values.astype(np.uint64, copy=False).reshape(values.shape[0], -1))
    values = [operator.index(v) for v in values]
    if any(v < 0 for v in values):
        raise ValueError("encoded values must be non-negative")
    return _lib.ints_to_limbs(values)


# Negative ints.  The reference's digit loops run on Python's two's-complement ints
# (``x & 3``, ``x >>= 2`` floor towards -inf), so where a loop ends, a negative input has an
# answer: TwoBit decode/gc_content read sequence_length digits (the value mod 4**L,
# encodings.py:97-99, 108-110); hamming_distance counts the digits of a ^ b, which is
# non-negative when both operands are negative (encodings.py:115-120); ThreeBit.decode
# reaches the all-ones top (triplet 7, not in its map) and raises KeyError at its lowest
# 0/5/7 triplet (encodings.py:177-178).  Where a loop never ends -- a negative XOR, a
# negative ThreeBit gc_content -- the drop-in raises ValueError instead of hanging.
_HANG_MIXED = ("hamming_distance of a negative and a non-negative code: their XOR is negative and the "
               "reference's `while difference:` loop (encodings.py:117, 198) never terminates on it")
_HANG_GC3 = ("ThreeBit.gc_content of a negative code: the reference's `while integer_encoded:` loop "
             "(encodings.py:189) never terminates on it")


def _twos_bits(v):
    """Bits that hold v in two's complement with its sign (non-negative: bit_length)."""
    return v.bit_length() if v >= 0 else (~v).bit_length() + 1


def _twos_limbs(values, words=None):
    """ints of any sign -> (n, words) limbs of v mod 2**(64 words): a negative value keeps its
    all-ones extension up to the top limb, so the XOR of two same-sign operands is exact."""
    if words is None:
        words = _lib.words_for_bits(max((_twos_bits(v) for v in values), default=0))
    m = (1 << (64 * words)) - 1
    return _lib.ints_to_limbs([v & m for v in values], words)


def _codes_mod(values, bits):
    """TwoBit decode/gc_content operands -> limbs; a negative int is read mod 2**bits."""
    if isinstance(values, np.ndarray) and values.dtype.kind in "ui":
        if values.dtype.kind == "i" and values.ndim == 1 and values.size and values.min() < 0:
            if bits <= 64:  # mod 2**64 keeps every digit the loop reads
                return values.astype(np.uint64).reshape(-1, 1)
            values = values.tolist()
        else:
            return _limbs_of(values)
    values = [operator.index(v) for v in values]
    if any(v < 0 for v in values):
        m = (1 << max(bits, 0)) - 1
        values = [v & m for v in values]
    return _lib.ints_to_limbs(values)


def _pair_limbs(a, b):
    """hamming_distance operands -> equal-width limbs whose XOR is a ^ b per pair."""
    def flat_ints(x):
        return (isinstance(x, np.ndarray) and x.dtype.kind in "ui"
                and (x.ndim == 1 or (x.ndim == 2 and x.shape[1] == 1)))
    if flat_ints(a) and flat_ints(b):
        a1, b1 = a.reshape(-1), b.reshape(-1)
        if a1.shape != b1.shape:
            raise ValueError("operand shapes differ: %s vs %s" % (a1.shape, b1.shape))
        na = a1 < 0 if a1.dtype.kind == "i" else np.zeros(a1.shape, bool)
        nb = b1 < 0 if b1.dtype.kind == "i" else np.zeros(b1.shape, bool)
        if (na != nb).any():
            raise ValueError(_HANG_MIXED)
        # same signs: the XOR of the uint64 views is the (non-negative) XOR of the ints (64-bit
        # arrays are viewed, not copied: a 100M-pair call moves 1.6 GB through the link anyway)
        def u64(x):
            x = np.ascontiguousarray(x)
            return x.view(np.uint64) if x.dtype.itemsize == 8 else x.astype(np.uint64)
        return u64(a1).reshape(-1, 1), u64(b1).reshape(-1, 1)
    if isinstance(a, np.ndarray) and a.ndim == 2 or isinstance(b, np.ndarray) and b.ndim == 2:
        la, lb = _limbs_of(a), _limbs_of(b)  # limb arrays: non-negative by construction
        w = max(la.shape[1], lb.shape[1])
        return _pad(la, w), _pad(lb, w)
    a = [operator.index(v) for v in (a.tolist() if isinstance(a, np.ndarray) else a)]
    b = [operator.index(v) for v in (b.tolist() if isinstance(b, np.ndarray) else b)]
    if len(a) != len(b):
        raise ValueError("operand shapes differ: (%d,) vs (%d,)" % (len(a), len(b)))
    if any((x < 0) != (y < 0) for x, y in zip(a, b)):
        raise ValueError(_HANG_MIXED)
    words = _lib.words_for_bits(max((_twos_bits(v) for v in a + b), default=0))
    return _twos_limbs(a, words), _twos_limbs(b, words)


def _three_lift(x):
    """A negative ThreeBit value -> the non-negative one that decodes to the same KeyError:
    its triplets up to the first all-ones (7) triplet of the sign extension."""
    top = -(-(~x).bit_length() // 3)  # first triplet lying wholly in the sign extension
    return x & ((1 << (3 * (top + 1))) - 1)


class Encoding:
    """Abstract base class for DNA encodings (encodings.py:4-33)."""

    encoding_map = NotImplemented
    decoding_map = NotImplemented
    bits_per_base = NotImplemented

    @classmethod
    def encode(cls, bytes_encoded):
        raise NotImplementedError

    def decode(self, integer_encoded):
        raise NotImplementedError

    def gc_content(self, integer_encoded):
        raise NotImplementedError

    @staticmethod
    def hamming_distance(a, b):
        raise NotImplementedError


class TwoBit(Encoding):
    """2-bit DNA encoding (encodings.py:36-121); ambiguous bases are randomised.

    :param int sequence_length: number of nucleotides that are being encoded
    """

    def __init__(self, sequence_length):
        self.sequence_length = sequence_length

    class TwoBitEncodingMap:
        """Read-only dict look-alike (encodings.py:53-69), kept for API parity."""

        map_ = dict(_VALID2)
        iupac_ambiguous = set(_AMBIGUOUS)

        def __getitem__(self, byte):
            try:
                return self.map_[byte]
            except KeyError:
                if byte not in self.iupac_ambiguous:
                    raise KeyError('%s is not a valid IUPAC nucleotide code' % chr(byte))
                return random.randint(0, 3)

    encoding_map = TwoBitEncodingMap()
    decoding_map = {0: b'A', 1: b'C', 2: b'T', 3: b'G'}
    bits_per_base = 2

    # ------------------------------------------------------------ batch API
    @classmethod
    def encode_array(cls, seqs, return_gc=False):
        """Encode equal-length records -> uint64 codes ((n,) if 2L <= 64 else (n, words)).

        Draws random numbers for ambiguous bases exactly as n calls of encode() would."""
        recs = _records(seqs)
        codes, gc, flags = _encode_records(2, recs)
        _fill_ambiguous(recs, codes, gc, flags)
        out = codes[:, 0] if codes.shape[1] == 1 else codes
        return (out, gc) if return_gc else out

    def decode_array(self, codes):
        """codes -> 'S<L>' array of decoded barcodes (encodings.py:90-100)."""
        limbs = _codes_mod(codes, 2 * self.sequence_length)
        raw = _lib.decode2(limbs, self.sequence_length)
        return raw.view("S%d" % max(1, self.sequence_length)).reshape(-1) if self.sequence_length else \
            np.array([b""] * limbs.shape[0], dtype="S1")

    def gc_content_array(self, codes):
        return _lib.gc_content(2, _codes_mod(codes, 2 * self.sequence_length), self.sequence_length)

    @staticmethod
    def hamming_distance_array(a, b):
        return _lib.hamming_pairs(2, *_pair_limbs(a, b))

    # ------------------------------------------------------------ reference API
    @classmethod
    def encode(cls, bytes_encoded):
        """encodings.py:75-88 (batch of one)."""
        code = _scalar.encode(2, bytes_encoded)  # a bytes record of one limb, no ambiguous base
        if code is not NotImplemented:
            return code
        if isinstance(bytes_encoded, str):
            if not bytes_encoded:
                return 0
            # the reference indexes its byte map with a str and then calls chr() on it
            raise TypeError("'str' object cannot be interpreted as an integer")
        seq = _as_bytes(bytes_encoded)
        if 0 < len(seq) <= 32:  # one limb: the lean scalar call
            code, flags = _lib.encode1(2, seq)
            if not flags:
                return code
        recs = np.frombuffer(seq, dtype=np.uint8).reshape(1, len(seq))
        codes, gc, flags = _lib.encode(2, recs, len(seq))
        _fill_ambiguous(recs, codes, gc, flags)
        return _lib.limbs_to_ints(codes)[0]

    def decode(self, integer_encoded):
        """encodings.py:90-100 (batch of one); a negative int reads mod 4**L there."""
        out = _scalar.decode2(integer_encoded, self.sequence_length)  # an int in [0, 2^64), 1 <= L <= 64
        if out is not NotImplemented:
            return out
        x = operator.index(integer_encoded)
        L = self.sequence_length
        if L <= 0:  # range(L) is empty
            return b''
        if x < 0:
            x &= (1 << (2 * L)) - 1
        if x < _U64 and L <= 64:
            return _lib.decode2_1(x, L)
        return _lib.decode2(_lib.ints_to_limbs([x]), L)[0].tobytes()

    def gc_content(self, integer_encoded):
        """encodings.py:102-111 (batch of one); a negative int reads mod 4**L there."""
        gc = _scalar.gc(2, integer_encoded, self.sequence_length)  # an int in [0, 2^64), L >= 1
        if gc is not NotImplemented:
            return gc
        x = operator.index(integer_encoded)
        L = self.sequence_length
        if L <= 0:
            return 0
        if x < 0:
            x &= (1 << (2 * L)) - 1
        if x < _U64:
            return _lib.gc1(2, x, L)
        return int(_lib.gc_content(2, _lib.ints_to_limbs([x]), L)[0])

    @staticmethod
    def hamming_distance(a, b):
        """encodings.py:113-121 (batch of one)."""
        d = _scalar.hamming(2, a, b)  # two ints in [0, 2^64)
        return _hamming1(2, a, b) if d is NotImplemented else d


class ThreeBit(Encoding):
    """3-bit DNA encoding (encodings.py:124-202); N stays distinct, length is implicit."""

    def __init__(self, *args, **kwargs):
        pass

    class ThreeBitEncodingMap:
        """encodings.py:139-149, kept for API parity."""

        map_ = {ord('C'): 1, ord('A'): 2, ord('G'): 3, ord('T'): 4, ord('N'): 6,
                ord('c'): 1, ord('a'): 2, ord('g'): 3, ord('t'): 4, ord('n'): 6}

        def __getitem__(self, byte):
            try:
                return self.map_[byte]
            except KeyError:
                return 6

    encoding_map = ThreeBitEncodingMap()
    decoding_map = {1: b'C', 2: b'A', 3: b'G', 4: b'T', 6: b'N'}
    bits_per_base = 3

    # ------------------------------------------------------------ batch API
    @classmethod
    def encode_array(cls, seqs, return_gc=False):
        recs = _records(seqs)
        codes, gc, _ = _encode_records(3, recs)
        out = codes[:, 0] if codes.shape[1] == 1 else codes
        return (out, gc) if return_gc else out

    @classmethod
    def decode_array(cls, codes):
        """codes -> list of bytes; raises KeyError like the reference on a bad triplet
        (every negative code has one: see _three_lift)."""
        if not (isinstance(codes, np.ndarray) and (codes.dtype.kind == "u" or codes.ndim == 2
                                                   or not codes.size or codes.min() >= 0)):
            codes = [operator.index(v) for v in (codes.tolist() if isinstance(codes, np.ndarray) else codes)]
            codes = [_three_lift(v) if v < 0 else v for v in codes]
        out, lengths, bad = _lib.decode3(_limbs_of(codes))
        res = []
        w = out.shape[1]
        for r in range(out.shape[0]):
            if bad[r] >= 0:
                raise KeyError(int(bad[r]))
            res.append(out[r, w - lengths[r]:].tobytes())
        return res

    @classmethod
    def gc_content_array(cls, codes):
        try:
            limbs = _limbs_of(codes)
        except ValueError:
            raise ValueError(_HANG_GC3) from None
        return _lib.gc_content(3, limbs)

    @staticmethod
    def hamming_distance_array(a, b):
        return _lib.hamming_pairs(3, *_pair_limbs(a, b))

    # ------------------------------------------------------------ reference API
    @classmethod
    def encode(cls, bytes_encoded):
        """encodings.py:155-167 (batch of one)."""
        code = _scalar.encode(3, bytes_encoded)  # a bytes record of one limb
        if code is not NotImplemented:
            return code
        if isinstance(bytes_encoded, str):
            # iterating a str yields str characters: none is in the byte map -> all N (6)
            seq = b"N" * len(bytes_encoded)
        else:
            seq = _as_bytes(bytes_encoded)
        if 0 < len(seq) <= 21:  # one limb: the lean scalar call
            return _lib.encode1(3, seq)[0]
        recs = np.frombuffer(seq, dtype=np.uint8).reshape(1, len(seq))
        codes, _, _ = _lib.encode(3, recs, len(seq))
        return _lib.limbs_to_ints(codes)[0]

    @classmethod
    def decode(cls, integer_encoded):
        """encodings.py:169-180 (batch of one)."""
        out = _scalar.decode3(integer_encoded)  # an int in [0, 2^64) whose triplets all decode
        return cls.decode_array([integer_encoded])[0] if out is NotImplemented else out

    @classmethod
    def gc_content(cls, integer_encoded):
        """encodings.py:182-192 (batch of one)."""
        gc = _scalar.gc(3, integer_encoded, 0)  # an int in [0, 2^64)
        if gc is not NotImplemented:
            return gc
        x = operator.index(integer_encoded)
        if x < 0:
            raise ValueError(_HANG_GC3)
        if x < _U64:
            return _lib.gc1(3, x)
        return int(_lib.gc_content(3, _lib.ints_to_limbs([x]))[0])

    @staticmethod
    def hamming_distance(a, b):
        """encodings.py:194-202 (batch of one)."""
        d = _scalar.hamming(3, a, b)  # two ints in [0, 2^64)
        return _hamming1(3, a, b) if d is NotImplemented else d


def _pad(limbs, words):
    if limbs.shape[1] == words:
        return limbs
    out = np.zeros((limbs.shape[0], words), dtype=np.uint64)
    out[:, :limbs.shape[1]] = limbs
    return out


def _hamming1(kind, a, b):
    a, b = operator.index(a), operator.index(b)
    if 0 <= a < _U64 and 0 <= b < _U64:
        return _lib.hamming1(kind, a, b)
    if (a < 0) != (b < 0):
        raise ValueError(_HANG_MIXED)
    words = _lib.words_for_bits(max(_twos_bits(a), _twos_bits(b)))
    if words == 1:  # both negative within int64: the uint64 views XOR to a ^ b
        return _lib.hamming1(kind, a & (_U64 - 1), b & (_U64 - 1))
    la, lb = _twos_limbs([a], words), _twos_limbs([b], words)
    return int(_lib.hamming_pairs(kind, la, lb)[0])
