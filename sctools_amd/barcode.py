"""Drop-in for ``sctools.barcode`` (src/sctools/barcode.py) on MI355X.

``Barcodes`` keeps the reference's Mapping semantics (code -> count, unique keys in
insertion order, barcode.py:8-37).  ``summarize_hamming_distances`` replaces the
O(n^2) Python pair loop (barcode.py:42-43) with the all-pairs HIP kernel, which
returns the exact distance histogram, and reproduces ``np.percentile``/``np.mean``
(barcode.py:44-46) bit-for-bit from that histogram in the library's host code.
The README's ``ObservedBarcodeSet`` / ``PriorBarcodeSet`` names (README.md:33) are
provided as subclasses.
"""

import itertools
from collections import Counter
from collections.abc import Mapping

import numpy as np

from . import _lib, _pykeys
from .encodings import TwoBit
from .stats import base4_entropy

__all__ = ["Barcodes", "ObservedBarcodeSet", "PriorBarcodeSet", "WhitelistCorrector", "nearest_whitelist"]

_MIXED_SIGNS = ('barcode codes mix negative and non-negative integers: their XOR is negative and the '
                'reference\'s distance loop (encodings.py:118, `while difference:`) never terminates on it')
_NEGATIVE_OUTSIDE = ('nearest needs non-negative barcode codes: a negative key has no TwoBit distance '
                     'to a non-negative query that the reference\'s distance loop (encodings.py:118) ends on')
_SUMMARY_KEYS = ('minimum', '25th percentile', 'median', '75th percentile', 'maximum', 'average')


class Barcodes:

    def __init__(self, barcodes, barcode_length):
        """Container for a set of barcodes encoded in 2-bit form (barcode.py:10-25).

        :param Mapping barcodes: dictionary mapping barcodes to counts
        :param int barcode_length: the length of all barcodes in the set
        """
        if not isinstance(barcodes, Mapping):
            raise TypeError('barcode set must be a dict-like object mapping barcodes to counts')
        self._data = barcodes
        # the reference's check (barcode.py:23-24) only fires for non-int lengths > 0
        if not isinstance(barcode_length, int) and barcode_length > 0:
            raise ValueError('barcode length must be a positive integer')
        self._barcode_length = barcode_length

    def __contains__(self, item):
        return item in self._data

    def __iter__(self):
        return iter(self._data)

    def __len__(self):
        return len(self._data)

    def __getitem__(self, item):
        return self._data[item]

    # ------------------------------------------------------------ device input
    def codes_array(self, mask_negative=True):
        """The unique keys in iteration order, as the kernels take them: np.uint64 (n,)
        when every key fits 64 bits, else (n, words) little-endian uint64 limbs.  Built from
        the mapping on every call (the reference re-reads ``self`` each time, barcode.py:42),
        so a mapping changed in place is never served stale.

        Negative keys: the reference's ``a ^ b`` of two negative ints is non-negative and its
        digit loop (encodings.py:113-121) counts it, so an all-negative key set is summarised
        like any other: every key shares its bits from m = max bit_length(~k) upward (all
        ones), so ``k & (2^m - 1)`` keeps every pairwise XOR unchanged.  A negative key next
        to a non-negative one gives a negative XOR, on which the reference's ``while
        difference:`` never ends; that raises ValueError here instead of hanging.  The masking
        only preserves XORs WITHIN the set, so callers comparing the codes with outside values
        (``nearest``) pass ``mask_negative=False`` and get ValueError for any negative key."""
        return self._codes_and_bits(mask_negative)[0]

    def _codes_and_bits(self, mask_negative=True):
        """codes_array() and, when the C key loop gave it for free, the bit length of the
        largest code (None otherwise: the library takes it from the codes)."""
        keys = self._data.keys()
        n = len(self._data)
        # the common case (Python-int keys within int64) in one C loop (csrc/pykeys.c): the type
        # check, the conversion and the keys' min / max together (no numpy pass over the codes
        # for the sign check or the width); every other case takes the general path below
        arr = np.empty(n, dtype=np.int64)
        status, got, lo, hi = _pykeys.keys_to_int64(self._data if type(self._data) in (dict, Counter) else keys, arr)
        if status == 0 and got == n:
            if lo >= 0:
                return arr.view(np.uint64), int(hi).bit_length()
            return self._finish_int64(arr, mask_negative), None
        if not all(issubclass(t, (int, np.integer)) for t in set(map(type, keys))):
            # the reference's pair loop dies at its first ``a ^ b`` on a non-integer key
            # (encodings.py:117 via barcode.py:42-43): raise exactly that TypeError
            for a, b in itertools.combinations(self._data, 2):
                a ^ b
            return np.zeros(n, dtype=np.uint64), None  # < 2 keys: no pair, nothing to compare
        try:  # numpy integer keys within int64
            return self._finish_int64(np.fromiter(keys, dtype=np.int64, count=n), mask_negative), None
        except OverflowError:
            pass
        if not any(isinstance(k, np.signedinteger) and k < 0 for k in keys):  # (numpy would wrap those)
            try:
                return np.fromiter(keys, dtype=np.uint64, count=n), None
            except OverflowError:
                pass
        ints = [int(k) for k in keys]
        neg = [v < 0 for v in ints]
        if any(neg):
            if not mask_negative:
                raise ValueError(_NEGATIVE_OUTSIDE)
            if not all(neg) and n >= 2:
                raise ValueError(_MIXED_SIGNS)
            mask = (1 << max((~v).bit_length() for v in ints)) - 1
            ints = [v & mask for v in ints]
        return _lib.ints_to_limbs(ints), None

    @staticmethod
    def _finish_int64(arr, mask_negative):
        """int64 keys -> the kernels' uint64 codes (negative keys: see codes_array)."""
        if arr.size and int(arr.min()) < 0:
            if not mask_negative:
                raise ValueError(_NEGATIVE_OUTSIDE)
            if int(arr.max()) >= 0 and arr.size >= 2:
                raise ValueError(_MIXED_SIGNS)
            m = int((~arr).max()).bit_length()
            return (arr & np.int64((1 << m) - 1)).view(np.uint64) if m < 63 else arr.view(np.uint64)
        return arr.view(np.uint64)

    def hamming_histogram(self):
        """np.uint64 histogram H[d] of TwoBit distances over all unordered pairs."""
        codes, bits = self._codes_and_bits()
        if codes.ndim == 2:  # keys >= 2^64: the multi-limb pair kernel
            hist = _lib.hamming_hist_allpairs_wide(codes)
        else:
            hist = _lib.hamming_hist_allpairs(codes, bits, distinct=True)  # mapping keys: distinct
        want = (self._barcode_length + 1) if isinstance(self._barcode_length, int) else 0
        if want > hist.size:  # bins up to the barcode length, as np.bincount(minlength=L+1)
            hist = np.concatenate([hist, np.zeros(want - hist.size, dtype=hist.dtype)])
        return hist

    def summarize_hamming_distances(self):
        """returns descriptive statistics on hamming distances between pairs of barcodes
        (barcode.py:39-46).

        From the SPECTRAL threshold (325K 16-bp codes) the count splits over every device of
        ``sctools_amd.set_devices()`` (default: all visible GPUs).  The call frees all the device
        memory it mapped before it returns (up to 4 GiB per device); with
        ``sctools_amd.keep_workspace(True)`` it stays cached for the next call instead."""
        hist = self.hamming_histogram()
        values = _lib.summary_from_hist(hist)  # IndexError for < 2 barcodes, as numpy raises
        return dict(zip(_SUMMARY_KEYS, [np.float64(v) for v in values]))

    def nearest(self, queries, max_distance=1):
        """For each TwoBit-encoded query, the index (in iteration order) of the unique
        closest barcode of this set within ``max_distance`` (TwoBit.hamming_distance),
        -2 for a tie, -1 for none; and that distance (255 for none)."""
        codes = self.codes_array(mask_negative=False)
        if codes.ndim != 1:
            raise ValueError('nearest needs barcode codes below 2**64')
        return nearest_whitelist(queries, codes, max_distance=max_distance, encoding='TwoBit')

    def base_frequency(self, weighted=False):
        """(barcode_length, 4) uint64 base counts by position, columns A, C, T, G
        (barcode.py:48-70)."""
        codes = np.fromiter(self._data.keys(), dtype=np.uint64)  # OverflowError >= 2^64, as there
        if weighted and self._barcode_length > 0:  # raised inside the position loop there (:66-67)
            raise NotImplementedError
        return _lib.base_frequency(codes, self._barcode_length)

    def effective_diversity(self, weighted=False):
        """Per-position base-4 entropy in [0, 1] (barcode.py:72-82)."""
        return base4_entropy(self.base_frequency(weighted=weighted))

    # ------------------------------------------------------------ constructors
    @classmethod
    def from_whitelist(cls, file_, barcode_length):
        """Barcode set from a whitelist file (barcode.py:84-97).

        As in the reference each line loses exactly its LAST byte (``barcode[:-1]``),
        every line is TwoBit-encoded, and duplicates collapse through Counter.  The file's
        bytes go to the GPU whole: the line split, the chop and the encode run there
        (sctools_amd/csrc/lines.hip); lines with ambiguous or invalid bytes are then redone
        in file order through TwoBit.encode, so the random draws and the KeyError of
        encodings.py:63-69 happen exactly as the reference's loop makes them."""
        with open(file_, 'rb') as f:
            data = f.read()
        codes, starts, lens, flags = _lib.whitelist_encode(data, 2)
        vals = codes[:, 0].tolist() if codes.shape[1] == 1 else _lib.limbs_to_ints(codes)
        for i in np.flatnonzero(flags).tolist():
            s = int(starts[i])
            vals[i] = TwoBit.encode(data[s:s + int(lens[i])])
        return cls(Counter(vals), barcode_length)

    @classmethod
    def from_iterable_encoded(cls, iterable, barcode_length):
        """construct an ObservedBarcodeSet from an iterable of encoded barcodes"""
        return cls(Counter(iterable), barcode_length=barcode_length)

    @classmethod
    def from_iterable_strings(cls, iterable, barcode_length):
        """construct an ObservedBarcodeSet from an iterable of string barcodes"""
        return cls(Counter(_encode_items(iterable, lambda b: _item_bytes(b.encode()))), barcode_length=barcode_length)

    @classmethod
    def from_iterable_bytes(cls, iterable, barcode_length):
        """construct an ObservedBarcodeSet from an iterable of bytes barcodes"""
        return cls(Counter(_encode_items(iterable, _item_bytes)), barcode_length=barcode_length)


def _encode_items(iterable, to_bytes):
    """TwoBit codes of ``to_bytes(item)`` for every item, in order, batched on the GPU.

    The reference takes item, converts, encodes, then the next item (barcode.py:104-114, a
    generator inside Counter).  So when an item's conversion fails -- or the iterable itself
    raises -- the items before it have already made their random draws, and an earlier item's
    KeyError surfaces instead: the items taken so far are encoded (draws and KeyError in record
    order) before the error is re-raised."""
    seqs = []
    try:
        for b in iterable:
            seqs.append(to_bytes(b))
    except Exception:
        _encode_lines(seqs)
        raise
    return _encode_lines(seqs)


def _item_bytes(b):
    """One from_iterable_bytes item as TwoBit.encode iterates it (encodings.py:85): bytes-like
    items as they are; any other iterable of byte values through bytes(); a non-iterable raises
    the reference's TypeError ("'int' object is not iterable"); a str raises the TypeError its
    characters raise in the byte map (an empty str encodes to 0)."""
    if isinstance(b, (bytes, bytearray, memoryview)):
        return bytes(b)
    if isinstance(b, str):
        if b:
            raise TypeError("'str' object cannot be interpreted as an integer")
        return b""
    return bytes(iter(b))


def _encode_lines(seqs):
    """TwoBit-encode a list of bytes in order; equal-length runs go to the GPU as one
    batch each, and ambiguous-base draws follow record order (see encodings.py)."""
    if not seqs:
        return []
    lengths = {len(s) for s in seqs}
    if len(lengths) == 1:
        codes = TwoBit.encode_array(seqs)
        return _lib.limbs_to_ints(codes.reshape(len(seqs), -1))
    # ragged input: per-length batches, but the random draws must follow record order,
    # so encode deterministic records in batches and walk the flagged ones in order.
    out = [None] * len(seqs)
    by_len = {}
    for i, s in enumerate(seqs):
        by_len.setdefault(len(s), []).append(i)
    pending = []
    for L, idx in by_len.items():
        recs = np.frombuffer(b"".join(seqs[i] for i in idx), dtype=np.uint8).reshape(len(idx), L)
        codes, _, flags = _lib.encode(2, recs, L)
        vals = _lib.limbs_to_ints(codes)
        for k, i in enumerate(idx):
            out[i] = vals[k]
            if flags[k]:
                pending.append(i)
    for i in sorted(pending):
        out[i] = TwoBit.encode(seqs[i])  # batch of one: draws in record order
    return out


class WhitelistCorrector:
    """``nearest_whitelist`` against one whitelist for a stream of query batches: the device
    index of the whitelist is built once, here, and every ``nearest(queries)`` call only copies
    its queries in and the results out (no reference counterpart).  The
    whitelist is copied at construction: changing the caller's array afterwards changes nothing.
    The index is built on every device of ``devices`` (default: ``sctools_amd.set_devices()``'s,
    every visible GPU) and each batch splits over them.

    :return of nearest (np.ndarray[int32], np.ndarray[uint8]): index, distance -- as
        ``nearest_whitelist``
    """

    def __init__(self, whitelist, max_distance=1, encoding='ThreeBit', devices=None):
        self.kind = {'ThreeBit': 3, 'TwoBit': 2, 3: 3, 2: 2}[encoding]
        self.max_distance = max_distance
        wl = np.ascontiguousarray(np.asarray(whitelist, dtype=np.uint64)).reshape(-1)
        self.size = wl.size
        self._plan = None
        if wl.size:
            bits = max(int(np.bitwise_or.reduce(wl)).bit_length(), self.kind * (max_distance + 1))
            self._plan = _lib.HostNearestPlan(self.kind, wl, min(64, bits), max_distance, devices=devices)

    def nearest(self, queries):
        q = np.ascontiguousarray(np.asarray(queries, dtype=np.uint64)).reshape(-1)
        if self._plan is None:
            return np.full(q.size, -1, np.int32), np.full(q.size, 255, np.uint8)
        return self._plan.query(q)

    def close(self):
        if self._plan is not None:
            self._plan.close()
            self._plan = None


def nearest_whitelist(queries, whitelist, max_distance=1, encoding='ThreeBit', devices=None):
    """Whitelist error correction (no reference counterpart).

    Same result as the brute force over the reference's distance
    (``ThreeBit.hamming_distance``, encodings.py:194-202, or ``TwoBit.hamming_distance``,
    encodings.py:113-121): for each query the unique whitelist index at the minimal
    distance d <= max_distance, -2 if several indices share it, -1 if none; plus d
    (255 when none).  Codes are non-negative ints below 2**64 in the given encoding.

    :return (np.ndarray[int32], np.ndarray[uint8]): index, distance
    """
    kind = {'ThreeBit': 3, 'TwoBit': 2, 3: 3, 2: 2}[encoding]
    wl = np.ascontiguousarray(np.asarray(whitelist, dtype=np.uint64)).reshape(-1)
    q = np.ascontiguousarray(np.asarray(queries, dtype=np.uint64)).reshape(-1)
    if wl.size == 0:
        return np.full(q.size, -1, np.int32), np.full(q.size, 255, np.uint8)
    bits = max(int(np.bitwise_or.reduce(wl)).bit_length(), kind * (max_distance + 1))
    return _lib.nearest(kind, wl, q, max_d=max_distance, code_bits=min(64, bits), devices=devices)


class ObservedBarcodeSet(Barcodes):
    """README.md:33 name for a set of observed barcodes (same behaviour as Barcodes)."""


class PriorBarcodeSet(Barcodes):
    """README.md:33 name for a set of expected (whitelist) barcodes."""
