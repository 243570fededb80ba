"""Drop-in for sctools.fastq's barcode extraction (src/sctools/fastq.py:159-200).

``EmbeddedBarcodeGenerator(embedded_barcodes, files, mode)`` yields, per FASTQ record,
``[(sequence_tag, record.sequence[start:end], 'Z'), (quality_tag, record.quality[start:end],
'Z'), ...]`` exactly as the reference does, but the record splitting and slicing of every
record happen in one pass on the GPU (sctools_amd/csrc/fastq.hip); Python objects are made
only for the records actually iterated.  ``extract_arrays()`` is the batch form that feeds
the hot path without per-record objects: fixed-width numpy rows plus lengths, ready for
``encodings.TwoBit.encode_array`` / ``ThreeBit.encode_array``; ``iter_arrays()`` yields the
same per piece of the files, which are read lazily in pieces of ``CHUNK_BYTES`` (a record
cut by a piece end is carried into the next piece, also across a file boundary), so a
billion-read stream never sits in host memory whole.  Text mode accepts ASCII only (the
device slices bytes; a non-ASCII text file raises ValueError: read it in 'rb' mode).

File handling follows reader.Reader (src/sctools/reader.py:15-85): a str or a list of str
filenames, modes 'r' (text: universal newlines, str fields) and 'rb' (bytes fields), and
.gz / .bz2 files opened through gzip / bz2 (decompression stays on the host).
"""

import bz2
import gzip
import itertools
import os
import queue
import threading
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


def _open_binary(name):
    """reader.py:64-71: .gz / .bz2 by suffix, else a plain file, always as bytes (the device
    applies the text-mode newline rules)."""
    if name.endswith('.gz'):
        return gzip.open(name, 'rb')
    if name.endswith('.bz2'):
        return bz2.open(name, 'rb')
    return open(name, 'rb')


#: bytes per piece handed to the device (the files are read lazily, piece by piece)
CHUNK_BYTES = 256 << 20


#: bytes in front of every piece buffer for the tail carried over from the previous piece
_HEADROOM = 1 << 20


class _PieceReader(threading.Thread):
    """Fills page-locked piece buffers from the files, one buffer ahead of the consumer: each
    buffer in `free` comes back through get() as (buffer, bytes read at [head, head + n), the
    file ends among them, whether every file is exhausted), or an exception raised while
    opening or reading (raised by the consumer in its turn).  The read releases the GIL.  The
    files are read in sequence, so a missing or unreadable file surfaces after the pieces of
    the files before it (reader.py:64-71 opens each file when it gets there)."""

    def __init__(self, files, buffers, head):
        super().__init__(name="sctools-fastq-reader", daemon=True)
        self._files = list(files)
        self._head = head
        self._halt = False
        self.free = queue.Queue()
        self.full = queue.Queue()
        for b in buffers:
            self.free.put(b)

    def get(self, block=True):
        return self.full.get(block)

    def run(self):
        f = None
        names = iter(self._files)
        try:
            last = False
            while not last:
                buf = self.free.get()
                if buf is None or self._halt:
                    return
                mv = memoryview(buf)[self._head:]
                n, ends, cap = 0, [], buf.size - self._head
                while n < cap:
                    if f is None:
                        name = next(names, None)
                        if name is None:
                            last = True
                            break
                        f = _open_binary(name)
                    got = f.readinto(mv[n:])
                    if not got:
                        f.close()
                        f = None
                        ends.append(n)
                        continue
                    n += got
                del mv
                self.full.put((buf, n, ends, last))
        except BaseException as e:  # (handed to the consumer)
            self.full.put(e)
        finally:
            if f is not None:
                f.close()

    def close(self):
        """Stop after the current read (a consumer that stops early): the thread holds its own
        references to any buffer it is still filling, so a block is never reused under it."""
        self._halt = True
        self.free.put(None)
        self.join(timeout=10.0)


class _ParallelPieceReader:
    """The same pieces as _PieceReader, for plain (uncompressed, existing) files: segment k of the
    concatenated files -- bytes [k cap, (k + 1) cap) -- is read with os.preadv by one of W workers
    (page-cache copies on W cores at once: one reading thread was the FASTQ -> nearest flow's
    ceiling), and get() hands the segments back in order.  Buffers go to segments in segment
    order (one worker at a time takes the next free buffer and the next segment number), so the
    segment the consumer waits for always holds a buffer.  File ends as _PieceReader reports
    them: a file ending exactly at a segment's end is that of the next segment, at 0.

    The files' sizes are taken when they are opened (a snapshot: the segments need them), where the
    sequential reader reads each file to its EOF when it gets there.  So a file still being appended
    to would give different records: the last segment checks every size again and raises OSError,
    after the records before it, when one changed."""

    def __init__(self, files, buffers, head, workers):
        self._head = head
        self._halt = False
        self._cap = buffers[0].size - head
        self._fds = []
        try:
            for name in files:
                self._fds.append(os.open(name, os.O_RDONLY))
        except BaseException:
            self._close_fds()
            raise
        sizes = [os.fstat(fd).st_size for fd in self._fds]
        self._sizes = sizes
        self._bounds = list(itertools.accumulate(sizes))  # the files' ends in the concatenation
        self._starts = [b - z for b, z in zip(self._bounds, sizes)]
        total = self._bounds[-1] if self._bounds else 0
        self._nseg = total // self._cap + 1  # (the last one short, possibly empty)
        self.free = queue.Queue()
        for b in buffers:
            self.free.put(b)
        self._take = threading.Lock()  # (a free buffer and the next segment number, together)
        self._k_next = 0
        self._cv = threading.Condition()
        self._done = {}
        self._next = 0
        self._threads = [threading.Thread(target=self._work, name="sctools-fastq-reader-%d" % w, daemon=True)
                         for w in range(max(1, min(workers, self._nseg)))]

    def start(self):
        for t in self._threads:
            t.start()

    def get(self, block=True):
        with self._cv:
            while self._next not in self._done:
                if not block:
                    raise queue.Empty
                self._cv.wait()
            item = self._done.pop(self._next)
            self._next += 1
            return item

    def _fill(self, buf, k):
        lo = k * self._cap
        hi = min(lo + self._cap, self._bounds[-1] if self._bounds else 0)
        mv = memoryview(buf)
        for fd, fs, fe in zip(self._fds, self._starts, self._bounds):
            a, b = max(lo, fs), min(hi, fe)
            while a < b:  # (preadv may return short)
                got = os.preadv(fd, [mv[self._head + a - lo:self._head + b - lo]], a - fs)
                if got <= 0:
                    raise OSError("short read of a FASTQ file (it changed while being read?)")
                a += got
        ends = [e - lo for e in self._bounds if lo <= e < lo + self._cap]
        if k == self._nseg - 1 and [os.fstat(fd).st_size for fd in self._fds] != self._sizes:
            raise OSError("a FASTQ file changed size while being read (the parallel reader reads the "
                          "sizes the files had when they were opened)")
        return buf, hi - lo, ends, k == self._nseg - 1

    def _work(self):
        while True:
            with self._take:
                buf = self.free.get()
                if buf is None or self._halt or self._k_next >= self._nseg:
                    return
                k = self._k_next
                self._k_next += 1
            try:
                item = self._fill(buf, k)
            except BaseException as e:  # (handed to the consumer in its turn)
                item = e
            with self._cv:
                self._done[k] = item
                self._cv.notify_all()
            if isinstance(item, BaseException):
                return

    def _close_fds(self):
        for fd in self._fds:
            os.close(fd)
        self._fds = []

    def close(self):
        self._halt = True
        for _ in self._threads:
            self.free.put(None)
        for t in self._threads:
            t.join(timeout=10.0)
        if not any(t.is_alive() for t in self._threads):
            self._close_fds()


#: worker threads of the parallel piece reader (plain files)
READ_WORKERS = 3


def _piece_reader(files, chunk_bytes, head):
    """The reader for these files: parallel positional reads for plain files that all exist,
    else one thread reading them in order (compressed files, stdin, or a missing file, whose
    error then comes after the pieces before it)."""
    files = list(files)
    plain = files and all(not f.endswith(('.gz', '.bz2')) and os.path.isfile(f) for f in files)
    if plain and READ_WORKERS > 1 and hasattr(os, "preadv"):
        try:
            # W + 2 buffers (W filling, one ready, one with the consumer) of half-size pieces: the
            # page-locked footprint stays near the sequential reader's two full-size buffers
            seg = chunk_bytes // 2 if chunk_bytes >= (2 << 20) else chunk_bytes
            bufs = [_lib.pinned.empty(head + seg, np.uint8) for _ in range(READ_WORKERS + 2)]
            return _ParallelPieceReader(files, bufs, head, READ_WORKERS)
        except OSError:
            pass  # (the sequential reader reports it in order)
    return _PieceReader(files, [_lib.pinned.empty(head + chunk_bytes, np.uint8) for _ in range(2)], head)


def _last_line_end(buf, have):
    """1 + the position of the last '\\n' in buf[:have] (0 if none), searching back from the end
    in growing windows (a piece's last line end is normally within its last record)."""
    w = 1 << 16
    hi = have
    while hi > 0:
        lo = max(0, hi - w)
        hits = np.flatnonzero(buf[lo:hi] == 10)
        if hits.size:
            return lo + int(hits[-1]) + 1
        hi = lo
        w <<= 1
    return 0


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

    def _pieces(self, qualities=True, chunk_bytes=None):
        """Read the files lazily (reader.py:56-85) in pieces of about `chunk_bytes`, cut after
        their last '\\n'; the device extracts each piece's complete records and says where
        the next piece starts (a record cut by the piece end is carried over, also across a
        file boundary).  Yields (first record number, nrecords, first bad-name record of the
        piece or -1, per-span arrays).

        A reader thread (`_PieceReader`) fills one page-locked buffer while the device and the
        caller work on the other, so the file reads overlap everything else; the device copies
        each piece by DMA in place, the next one (when read already) while the caller works on
        this one's results (sct_fastq_stream_stage).  The carried-over tail goes into the headroom in front of
        the next piece (a tail longer than the headroom -- a record longer than a megabyte --
        is merged with the next piece in a new buffer)."""
        chunk_bytes = max(1, int(chunk_bytes or CHUNK_BYTES))
        head = _HEADROOM
        st = _lib.FastqStream([(eb.start, eb.end) for eb in self.embedded_barcodes], self._mode == 'r', qualities)
        reader = _piece_reader(self._files, chunk_bytes, head)
        reader.start()
        carry = np.zeros(0, np.uint8)  # the unconsumed tail of the last piece (a copy)
        carry_ends = []                # file ends inside it

        def prepare(got):
            """A segment from the reader -> (piece, file ends in it, last?, buffer to hand back,
            bytes of the chunk call to come: the cut after the last '\\n', the whole final piece)."""
            buf, n, seg_ends, last = got
            c = carry.size
            if c <= head:  # the tail goes in front of the segment, in the same buffer
                buf[head - c:head] = carry
                piece = buf[head - c:head + n]
                release = buf
            else:  # (a tail longer than the headroom: one merged buffer)
                piece = _lib.pinned.empty(c + n, np.uint8)
                piece[:c] = carry
                piece[c:] = buf[head:head + n]
                reader.free.put(buf)
                release = None
            ends = carry_ends + [c + e for e in seg_ends]
            return piece, ends, last, release, (piece.size if last else _last_line_end(piece, piece.size))

        done = 0
        nxt, pending = None, None
        try:
            while True:
                if nxt is None:
                    got = reader.get()
                    if isinstance(got, BaseException):
                        raise got
                    nxt = prepare(got)
                piece, ends, last, release, cut = nxt
                nxt = None
                if last:
                    nrec, _, bad, parts = st.chunk(piece, piece.size, ends or [0], final=True)
                    yield done, nrec, bad, parts
                    return
                used, out = 0, None
                if cut > 0:
                    nrec, used, bad, parts = st.chunk(piece, cut, [e for e in ends if e < cut] + [cut], final=False)
                    out = (done, nrec, bad, parts)
                carry = piece[used:].copy()  # (no line end, or no complete record yet: all of it)
                carry_ends = [e - used for e in ends if e > used]
                del piece
                if release is not None:
                    reader.free.put(release)
                if out is not None and out[2] < 0:
                    # the next piece, when the reader has it, goes to the device now: its copy then
                    # overlaps the caller's work on this piece's results
                    try:
                        got = reader.get(block=False)
                    except queue.Empty:
                        got = None
                    if isinstance(got, BaseException):
                        pending = got
                    elif got is not None:
                        nxt = prepare(got)
                        if nxt[4] > 0:
                            st.stage(nxt[0], nxt[4])
                if out is not None:
                    yield out
                    if out[2] >= 0:
                        return
                    done += out[1]
                if pending is not None:
                    raise pending
        finally:
            reader.close()
            st.close()

    def _run(self, qualities=True):
        """All records at once (the batch form): (nrecords, first bad record or -1, per-span
        arrays concatenated over the pieces)."""
        total, first_bad, acc = 0, -1, None
        for base, n, bad, parts in self._pieces(qualities):
            if acc is None:
                acc = [[[] for _ in range(4)] for _ in parts]
            for k, tup in enumerate(parts):
                for i, a in enumerate(tup):
                    if a is not None:
                        acc[k][i].append(a[: (bad if bad >= 0 else n)])
            if bad >= 0:
                return base + bad, base + bad, self._join(acc, qualities)
            total = base + n
        return total, first_bad, self._join(acc, qualities)

    def _join(self, acc, qualities):
        out = []
        for k, eb in enumerate(self.embedded_barcodes):
            w = eb.end - eb.start
            lists = acc[k] if acc is not None else [[] for _ in range(4)]
            cat = [np.concatenate(x) if x else None for x in lists]
            seq = cat[0] if cat[0] is not None else np.zeros((0, w), np.uint8)
            slen = cat[1] if cat[1] is not None else np.zeros(0, np.int32)
            qual = (cat[2] if cat[2] is not None else np.zeros((0, w), np.uint8)) if qualities else None
            qlen = (cat[3] if cat[3] is not None else np.zeros(0, np.int32)) if qualities else None
            out.append((seq, slen, qual, qlen))
        return out

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
        """reader.py:47-54 iterates every record, so a bad name line raises there too
        (fastq.py:35-36)."""
        total = 0
        for base, n, bad, _ in self._pieces(False):
            if bad >= 0:
                raise ValueError('fastq name must start with @')
            total = base + n
        return total

    def iter_arrays(self, qualities=True, chunk_bytes=None):
        """Streaming batch form: per piece of the files, the extract_arrays dict of that
        piece's records (a billion-read stream never sits in host memory whole)."""
        for base, n, bad, parts in self._pieces(qualities, chunk_bytes):
            stop = n if bad < 0 else bad
            out = {}
            for eb, (seq, slen, qual, qlen) in zip(self.embedded_barcodes, parts):
                w = eb.end - eb.start
                out[eb.sequence_tag] = (np.ascontiguousarray(seq[:stop]).view('S%d' % w).reshape(stop) if w else
                                        np.zeros(stop, dtype='S1'), slen[:stop])
                if qualities:
                    out[eb.quality_tag] = (np.ascontiguousarray(qual[:stop]).view('S%d' % w).reshape(stop) if w else
                                           np.zeros(stop, dtype='S1'), qlen[:stop])
            yield out
            if bad >= 0:
                raise ValueError('fastq name must start with @')

    def __iter__(self):
        text = self._mode == 'r'
        for base, n, bad, parts in self._pieces(True):
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
