"""Drop-in for sctools.fastq's barcode extraction (src/sctools/fastq.py:159-200).

``EmbeddedBarcodeGenerator(embedded_barcodes, files, mode)`` yields, per FASTQ record,
``[(sequence_tag, record.sequence[start:end], 'Z'), (quality_tag, record.quality[start:end],
'Z'), ...]`` exactly as the reference does, but the record splitting and slicing of every
record happen in one pass on the GPU (sctools_amd/csrc/fastq.hip); Python objects are made
only for the records actually iterated.  ``extract_arrays()`` is the batch form that feeds
the hot path without per-record objects: fixed-width numpy rows plus lengths, ready for
``encodings.TwoBit.encode_array`` / ``ThreeBit.encode_array``.

File handling follows reader.Reader (src/sctools/reader.py:15-85): a str or a list of str
filenames, modes 'r' (text: universal newlines, str fields) and 'rb' (bytes fields), and
.gz / .bz2 files opened through gzip / bz2 (decompression stays on the host).
"""

import bz2
import gzip
from collections import namedtuple
from collections.abc import Iterable

import numpy as np

from . import _lib

__all__ = ["EmbeddedBarcode", "EmbeddedBarcodeGenerator"]

# fastq.py:159 -- same field order and typename
EmbeddedBarcode = namedtuple('Tag', ['start', 'end', 'sequence_tag', 'quality_tag'])


def _filenames(files):
    """reader.py:21-31"""
    if isinstance(files, str):
        return [files]
    if isinstance(files, Iterable):
        files = list(files)
        if all(isinstance(f, str) for f in files):
            return files
        raise TypeError('all passed files must be type str')
    raise TypeError('files must be a string filename or a list of such names.')


def _read_bytes(name):
    """reader.py:64-71: .gz / .bz2 by suffix, else a plain file (bytes; the device applies
    the text-mode newline rules)."""
    if name.endswith('.gz'):
        with gzip.open(name, 'rb') as f:
            return f.read()
    if name.endswith('.bz2'):
        with bz2.open(name, 'rb') as f:
            return f.read()
    with open(name, 'rb') as f:
        return f.read()


class EmbeddedBarcodeGenerator:
    """fastq.py:165-200 on the device.  ``embedded_barcodes``: EmbeddedBarcode tuples with
    non-negative int start <= end."""

    def __init__(self, embedded_barcodes, files='-', mode='r'):
        self._files = _filenames(files)
        if mode not in {'r', 'rb'}:                              # reader.py:34-35
            raise ValueError('mode must be one of r, rb')
        self._mode = mode
        self.embedded_barcodes = list(embedded_barcodes)
        for eb in self.embedded_barcodes:
            if not (isinstance(eb.start, int) and isinstance(eb.end, int) and 0 <= eb.start <= eb.end):
                raise ValueError('EmbeddedBarcode start/end must be ints with 0 <= start <= end '
                                 'on the device path (got %r)' % (eb,))

    @property
    def filenames(self):
        return self._files

    def _run(self, qualities=True):
        blobs = [_read_bytes(f) for f in self._files]
        ends = np.cumsum([len(b) for b in blobs], dtype=np.int64)
        spans = [(eb.start, eb.end) for eb in self.embedded_barcodes]
        return _lib.fastq_extract(b''.join(blobs), ends, spans, self._mode == 'r', qualities)

    def extract_arrays(self, qualities=True):
        """Batch form: {sequence_tag: (rows 'S{w}', lengths), quality_tag: (...)} over every
        record.  Raises ValueError (the reference's message) if a record's name line does
        not start with '@'."""
        n, bad, parts = self._run(qualities)
        if bad >= 0:
            raise ValueError('fastq name must start with @')
        out = {}
        for eb, (seq, slen, qual, qlen) in zip(self.embedded_barcodes, parts):
            w = eb.end - eb.start
            out[eb.sequence_tag] = (np.ascontiguousarray(seq).view('S%d' % w).reshape(n) if w else
                                    np.zeros(n, dtype='S1'), slen.copy())
            if qualities:
                out[eb.quality_tag] = (np.ascontiguousarray(qual).view('S%d' % w).reshape(n) if w else
                                       np.zeros(n, dtype='S1'), qlen.copy())
        return out

    def __len__(self):
        """reader.py:47-54 counts lines; fastq records = lines // 4 (the grouper's zip)."""
        return self._run(False)[0]

    def __iter__(self):
        n, bad, parts = self._run(True)
        text = self._mode == 'r'
        stop = n if bad < 0 else bad
        for r in range(stop):
            rec = []
            for eb, (seq, slen, qual, qlen) in zip(self.embedded_barcodes, parts):
                s = bytes(seq[r, :slen[r]])
                q = bytes(qual[r, :qlen[r]])
                if text:
                    s, q = s.decode('ascii'), q.decode('ascii')
                rec.extend(((eb.sequence_tag, s, 'Z'), (eb.quality_tag, q, 'Z')))
            yield rec
        if bad >= 0:                                                  # fastq.py:35-36
            raise ValueError('fastq name must start with @')
