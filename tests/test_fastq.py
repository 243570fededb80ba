"""FASTQ embedded-barcode extraction (sctools_amd.fastq, csrc/fastq.hip) against the
reference's EmbeddedBarcodeGenerator outputs (tests/golden/fastq_golden.json, made by
tests/golden/gen_fastq_golden.py from the reference's own test FASTQs and edge cases)."""

import gzip
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN_DIR
from sctools_amd import encodings, fastq, platform

FQ_DIR = os.path.join(GOLDEN_DIR, "fastq")


@pytest.fixture(scope="module")
def fq_golden():
    with open(os.path.join(GOLDEN_DIR, "fastq_golden.json")) as f:
        return json.load(f)


def _ebs(g, tags):
    return [fastq.EmbeddedBarcode(start=s, end=e, sequence_tag=st, quality_tag=qt)
            for s, e, st, qt in (g["tags"][t] for t in tags)]


def _expected(records):
    out = []
    for rec in records:
        out.append([(t, v["str"] if isinstance(v, dict) else bytes.fromhex(v), z) for t, v, z in rec])
    return out


def _paths(case, tmp_path):
    if "files" in case:
        return [os.path.join(FQ_DIR, f) for f in case["files"]]
    paths = []
    for k, c in enumerate(case["contents"]):
        p = tmp_path / ("%s_%d.fastq" % (case["name"], k))
        p.write_bytes(bytes.fromhex(c))
        paths.append(str(p))
    return paths


# ---------------------------------------------------------------- CPU: argument handling
def test_reader_argument_errors():
    eb = [platform.TenXV2.cell_barcode]
    with pytest.raises(TypeError):
        fastq.EmbeddedBarcodeGenerator(eb, 10)
    with pytest.raises(TypeError):
        fastq.EmbeddedBarcodeGenerator(eb, ("works", 10))
    with pytest.raises(ValueError):
        fastq.EmbeddedBarcodeGenerator(eb, "works", "not_acceptable_open_mode")
    assert fastq.EmbeddedBarcode(0, 16, "CR", "CY")._fields == ("start", "end", "sequence_tag",
                                                                "quality_tag")


def test_golden_covers_reference_fixtures(fq_golden):
    names = {c["name"] for c in fq_golden["cases"]}
    assert {"test_r1.fastq", "test_i7.fastq", "short_reads", "crlf", "bad_name"} <= names
    assert fq_golden["tags"]["cell"] == [0, 16, "CR", "CY"]  # platform.py:36


# ---------------------------------------------------------------- GPU parity
@pytest.mark.gpu
def test_fastq_golden_cases(fq_golden, tmp_path):
    for case in fq_golden["cases"]:
        gen = fastq.EmbeddedBarcodeGenerator(_ebs(fq_golden, case["tags"]), _paths(case, tmp_path),
                                             case["mode"])
        got = []
        if "error" in case:
            with pytest.raises(ValueError) as ei:
                for rec in gen:
                    got.append(rec)
            assert str(ei.value) == case["error"]["args"][0]
        else:
            got = list(gen)
        assert got == _expected(case["records"]), (case["name"], case["mode"])


@pytest.mark.gpu
def test_fastq_gzip_and_batch_arrays(fq_golden, tmp_path):
    case = next(c for c in fq_golden["cases"] if c["name"] == "test_r1.fastq" and c["mode"] == "rb")
    raw = open(os.path.join(FQ_DIR, "test_r1.fastq"), "rb").read()
    gz = tmp_path / "r1.fastq.gz"
    gz.write_bytes(gzip.compress(raw))
    ebs = list(platform.TenXV2._tags["r1"])
    gen = fastq.EmbeddedBarcodeGenerator(ebs, str(gz), "rb")
    assert list(gen) == _expected(case["records"])
    assert len(gen) == 100
    arr = gen.extract_arrays()
    want = _expected(case["records"])
    assert [bytes(x) for x in arr["CR"][0]] == [r[0][1] for r in want]
    assert [bytes(x) for x in arr["UY"][0]] == [r[3][1] for r in want]
    assert arr["CR"][1].tolist() == [16] * 100
    # straight into the encoder: ThreeBit of the cell barcodes (N kept distinct)
    codes = encodings.ThreeBit.encode_array(arr["CR"][0])
    assert [int(c) for c in codes] == [encodings.ThreeBit.encode(r[0][1]) for r in want]


@pytest.mark.gpu
def test_fastq_synthetic_large_text_vs_python(tmp_path):
    """A 200k-record file with ragged reads and CRLF lines: the device slices equal a plain
    Python reading of the same file with the reference's line/slice rules."""
    rng = np.random.default_rng(5)
    lines = []
    for r in range(200_000):
        L = int(rng.integers(0, 40))
        seq = bytes(rng.choice(list(b"ACGTN"), size=L).tolist())
        nl = b"\r\n" if r % 7 == 0 else b"\n"
        lines += [b"@r%d" % r + nl, seq + nl, b"+" + nl, bytes([70] * L) + nl]
    blob = b"".join(lines)
    p = tmp_path / "big.fastq"
    p.write_bytes(blob)
    eb = [platform.TenXV2.cell_barcode, platform.TenXV2.molecule_barcode]
    for mode in ("rb", "r"):
        arr = fastq.EmbeddedBarcodeGenerator(eb, str(p), mode).extract_arrays()
        with open(p, mode) as f:
            py = f.readlines()
        seqs = py[1::4]
        for tag, (s, e) in (("CR", (0, 16)), ("UR", (16, 24))):
            want = [x[s:e] if mode == "rb" else x[s:e].encode() for x in seqs]
            rows, lens = arr[tag]
            assert lens.tolist() == [len(w) for w in want]
            assert [bytes(x) for x in rows] == want, (mode, tag)  # 'S' rows: NUL padding dropped


# ---------------------------------------------------------------- streaming (pieces)
class _FakeStream:
    """A host stand-in for sct_fastq_stream with the device's record rules (lines end at '\\n'
    and at file ends; records are 4 lines over all files; a non-final piece reports the bytes
    of its complete records), so the piece logic of _pieces -- the read-ahead thread, the
    carried tail, the file ends -- is checked on the CPU against one whole-input call."""

    staged_hits = 0

    def __init__(self, spans, text_mode, qualities=True):
        self.spans, self.qualities = [tuple(x) for x in spans], qualities
        self.staged = None

    def stage(self, buf, nbytes):
        """sct_fastq_stream_stage's contract, checked: the staged bytes must be unchanged when the
        chunk call for the same buffer and size comes."""
        a = np.asarray(buf)
        self.staged = (a.ctypes.data, nbytes, bytes(a[:nbytes]))

    def chunk(self, buf, nbytes, file_ends, final):
        data = bytes(np.asarray(buf)[:nbytes])
        if self.staged is not None:
            if self.staged[:2] == (np.asarray(buf).ctypes.data, nbytes):
                assert self.staged[2] == data, "a staged piece changed before its chunk call"
                _FakeStream.staged_hits += 1
            self.staged = None
        cuts = sorted(set([e for e in file_ends if 0 < e <= nbytes]))
        lines, pos = [], 0  # (start, end without '\\n', next start)
        while pos < nbytes:
            nl = data.find(b"\n", pos)
            stop = min([c for c in cuts if c > pos] + [nbytes])
            if nl < 0 or nl >= stop:
                if stop < nbytes or final or stop in cuts:
                    lines.append((pos, stop, stop))
                pos = stop
                continue
            lines.append((pos, nl, nl + 1))
            pos = nl + 1
        nrec = len(lines) // 4
        used = lines[4 * nrec - 1][2] if nrec else 0
        bad = next((r for r in range(nrec) if data[lines[4 * r][0]:lines[4 * r][0] + 1] != b"@"), -1)
        parts = []
        for a, b in self.spans:
            w = b - a
            seq = np.zeros((nrec, w), np.uint8)
            qual = np.zeros((nrec, w), np.uint8)
            sl = np.zeros(nrec, np.int32)
            ql = np.zeros(nrec, np.int32)
            for r in range(nrec):
                for li, arr, ln in ((1, seq, sl), (3, qual, ql)):
                    st, en, _ = lines[4 * r + li]
                    x = data[st:en][a:b]
                    arr[r, :len(x)] = np.frombuffer(x, np.uint8)
                    ln[r] = len(x)
            parts.append((seq, sl, qual if self.qualities else None, ql if self.qualities else None))
        return nrec, (nbytes if final else used), bad, parts

    def close(self):
        pass


@pytest.mark.parametrize("chunk", [5, 23, 64, 1000, 1 << 16])
def test_pieces_reader_carry_and_file_ends(tmp_path, monkeypatch, chunk):
    """_pieces in pieces of `chunk` bytes (tails longer than the headroom when the headroom is
    shrunk below a record) across files that cut records between any two lines, an empty file and a last file
    with no final newline: the records, their order and the per-piece counts equal one call over
    the whole input (host stand-in for the device: see _FakeStream)."""
    rng = np.random.default_rng(chunk)
    recs = []
    for r in range(400):
        L = int(rng.integers(0, 40))
        recs += [b"@r%d\n" % r, bytes(rng.choice(list(b"ACGTN"), size=L).tolist()) + b"\n", b"+\n",
                 bytes([70] * L) + b"\n"]
    blob = b"".join(recs)
    starts = np.cumsum([len(x) for x in recs])[:-1]  # files end between lines (inside records)
    bounds = sorted(set(rng.choice(starts, 4).tolist()))
    parts = [blob[i:j] for i, j in zip([0] + bounds, bounds + [len(blob)])]
    parts.insert(2, b"")  # an empty file
    parts[-1] = parts[-1][:-1]  # the last file has no final newline
    paths = []
    for k, part in enumerate(parts):
        p = tmp_path / ("p%d.fastq" % k)
        p.write_bytes(part)
        paths.append(str(p))
    monkeypatch.setattr(fastq._lib, "FastqStream", _FakeStream)
    if chunk <= 64:
        monkeypatch.setattr(fastq, "_HEADROOM", 8)  # tails outgrow the headroom: merged buffers
    eb = [fastq.EmbeddedBarcode(0, 16, "CR", "CY"), fastq.EmbeddedBarcode(4, 9, "UR", "UY")]
    gen = fastq.EmbeddedBarcodeGenerator(eb, paths, "rb")
    got = list(gen._pieces(True, chunk))
    # the whole input in one call, file ends at the files' ends
    ends, acc = [], 0
    for part in parts:
        acc += len(part)
        ends.append(acc)
    whole = np.frombuffer(b"".join(parts), np.uint8)
    n, _, bad, want = _FakeStream([(0, 16), (4, 9)], False).chunk(whole, whole.size, ends, True)
    if chunk <= 1000 and chunk != 64:
        assert _FakeStream.staged_hits > 0  # (the reader runs ahead: most pieces were staged)
    assert bad == -1 and n >= 399  # (399 when the last record's empty quality line was its final newline)
    assert sum(g[1] for g in got) == n
    assert [g[0] for g in got] == list(np.cumsum([0] + [g[1] for g in got[:-1]]))
    for k in range(2):
        for i in range(4):
            cat = np.concatenate([g[3][k][i] for g in got])
            assert np.array_equal(cat, want[k][i]), (k, i)


def test_pieces_reader_stops_when_abandoned(tmp_path, monkeypatch):
    """A consumer that stops after the first piece: closing the generator stops the reader
    threads (no thread left reading, the files closed), for the parallel and the in-order reader."""
    import threading
    p = tmp_path / "a.fastq"
    p.write_bytes(b"@a\nACGTACGTAC\n+\nFFFFFFFFFF\n" * 5000)
    gz = tmp_path / "a.fastq.gz"
    gz.write_bytes(gzip.compress(p.read_bytes()))
    monkeypatch.setattr(fastq._lib, "FastqStream", _FakeStream)
    for path in (p, gz):
        gen = fastq.EmbeddedBarcodeGenerator([fastq.EmbeddedBarcode(0, 4, "CR", "CY")], [str(path)], "rb")
        it = gen._pieces(True, 4096)
        first = next(it)
        assert first[1] > 0
        it.close()
        alive = [t for t in threading.enumerate() if t.name.startswith("sctools-fastq-reader")]
        assert not alive, alive


def test_pieces_reader_propagates_open_errors(tmp_path, monkeypatch):
    """A missing file raises FileNotFoundError from the generator (after the pieces before it)."""
    p = tmp_path / "a.fastq"
    p.write_bytes(b"@a\nACGT\n+\nFFFF\n" * 100)
    monkeypatch.setattr(fastq._lib, "FastqStream", _FakeStream)
    gen = fastq.EmbeddedBarcodeGenerator([fastq.EmbeddedBarcode(0, 4, "CR", "CY")],
                                         [str(p), str(tmp_path / "missing.fastq")], "rb")
    with pytest.raises(FileNotFoundError):
        list(gen._pieces(True, 64))


def test_parallel_reader_detects_a_growing_file(tmp_path):
    """The parallel reader reads the sizes the files had when opened; a file appended to while it
    reads is reported (OSError on the last segment), not silently cut."""
    p = tmp_path / "a.fastq"
    p.write_bytes(b"@a\nACGT\n+\nFFFF\n" * 1000)
    bufs = [np.zeros(64 + 4096, np.uint8) for _ in range(4)]
    r = fastq._ParallelPieceReader([str(p)], bufs, 64, 1)
    try:
        with open(p, "ab") as f:  # grows before the reader reaches its last segment
            f.write(b"@b\nACGT\n+\nFFFF\n")
        r.start()
        items = []
        while True:
            it = r.get()
            if isinstance(it, BaseException):
                items.append(it)
                break
            items.append(it)
            r.free.put(it[0])
            if it[3]:
                break
        assert isinstance(items[-1], OSError) and "changed size" in str(items[-1])
    finally:
        r.close()


def test_last_line_end_windows():
    """The piece cut: 1 + the last '\\n' in buf[:have], found back from the end in growing windows."""
    buf = np.full(300_000, ord("A"), np.uint8)
    assert fastq._last_line_end(buf, buf.size) == 0
    buf[5] = 10
    assert fastq._last_line_end(buf, buf.size) == 6  # (found in the widest window)
    buf[250_000] = 10
    assert fastq._last_line_end(buf, buf.size) == 250_001
    assert fastq._last_line_end(buf, 250_000) == 6  # (a '\\n' at or past `have` is not seen)
    assert fastq._last_line_end(buf, 0) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("chunk", [7, 64, 333])
def test_fastq_golden_cases_in_small_pieces(fq_golden, tmp_path, monkeypatch, chunk):
    """The files read lazily in tiny pieces (records and CRLF lines cut by piece ends, pieces
    spanning file boundaries): the same records and errors as the reference."""
    monkeypatch.setattr(fastq, "CHUNK_BYTES", chunk)
    test_fastq_golden_cases(fq_golden, tmp_path)


@pytest.mark.gpu
def test_fastq_len_raises_on_bad_name(fq_golden, tmp_path):
    case = next(c for c in fq_golden["cases"] if "error" in c)
    gen = fastq.EmbeddedBarcodeGenerator(_ebs(fq_golden, case["tags"]), _paths(case, tmp_path), case["mode"])
    with pytest.raises(ValueError) as ei:
        len(gen)
    assert str(ei.value) == "fastq name must start with @"


@pytest.mark.gpu
def test_fastq_multifile_stream_vs_python(tmp_path):
    """Three files (records spanning the file boundaries, the last file unterminated), read
    in 1 MB pieces and as one piece: identical arrays, equal to a plain Python reading of
    the concatenated lines; iter_arrays' pieces concatenate to the same."""
    rng = np.random.default_rng(9)
    lines = []
    for r in range(60_000):
        L = int(rng.integers(10, 60))
        seq = bytes(rng.choice(list(b"ACGTN"), size=L).tolist())
        lines += [b"@q%d\n" % r, seq + b"\n", b"+\n", bytes([65 + r % 20] * L) + b"\n"]
    # files cut between lines 2 and 3 / 1 and 2 of a record: records span the file ends
    c0, c1 = 4 * 20_000 + 2, 4 * 41_000 + 1
    parts = [b"".join(lines[:c0]), b"".join(lines[c0:c1]), b"".join(lines[c1:])[:-1]]  # last: no '\n'
    paths = []
    for k, part in enumerate(parts):
        p = tmp_path / ("s%d.fastq" % k)
        p.write_bytes(part)
        paths.append(str(p))
    eb = [platform.TenXV2.cell_barcode, platform.TenXV2.molecule_barcode]
    py_lines = []
    for p in paths:
        with open(p, "rb") as f:
            py_lines += f.readlines()
    seqs, quals = py_lines[1::4], py_lines[3::4]
    n = len(py_lines) // 4
    gen = fastq.EmbeddedBarcodeGenerator(eb, paths, "rb")
    whole = gen.extract_arrays()
    fastq_chunk = fastq.CHUNK_BYTES
    try:
        fastq.CHUNK_BYTES = 1 << 20
        small = gen.extract_arrays()
        assert len(gen) == n
        pieces = list(gen.iter_arrays())
    finally:
        fastq.CHUNK_BYTES = fastq_chunk
    assert len(pieces) > 3
    for tag, (s, e), src in (("CR", (0, 16), seqs), ("UY", (16, 24), quals)):
        want = [x[s:e] for x in src[:n]]
        for arr in (whole, small):
            rows, lens = arr[tag]
            assert rows.shape[0] == n and lens.tolist() == [len(w) for w in want]
            assert [bytes(x) for x in rows] == want
        cat = np.concatenate([p[tag][0] for p in pieces])
        assert cat.tolist() == whole[tag][0].tolist()


# ---------------------------------------------------------------- whitelist ingest
@pytest.mark.gpu
def test_whitelist_lines_on_device_vs_python(tmp_path):
    """from_whitelist's device line split + [:-1] chop + encode against Python's own line
    iteration of the same file (barcode.py:96-97), with ragged and empty lines and no final
    newline; a 737,280-line whitelist file as well."""
    from oracle import oracle as O
    from sctools_amd import barcode, synthetic
    rng = np.random.default_rng(12)
    lines = [bytes(rng.choice(list(b"ACGTacgt"), size=int(rng.integers(1, 40))).tolist()) + b"\n"
             for _ in range(5000)]
    lines[10] = b"\n"
    lines[4999] = lines[4999][:-1]
    p = tmp_path / "wl.txt"
    p.write_bytes(b"".join(lines))
    b = barcode.Barcodes.from_whitelist(str(p), 16)
    with open(p, "rb") as f:
        want = [O.two_bit_encode(ln[:-1]) for ln in f]
    from collections import Counter
    assert list(b) == list(Counter(want)) and [b[k] for k in b] == list(Counter(want).values())
    n, L, seed = synthetic.CONFIGS[2]
    codes = synthetic.whitelist_codes(n, L, seed)
    p2 = tmp_path / "737k.txt"
    p2.write_bytes(b"".join(r.tobytes() + b"\n" for r in synthetic.decode_ascii(codes, L)))
    big = barcode.PriorBarcodeSet.from_whitelist(str(p2), L)
    assert np.array_equal(big.codes_array(), codes)


def _fused(data, ends, spans, text_mode, cap=None, encode=True, kind=2):
    """sct_fastq_extract_fused on device copies; returns (nrec, first_bad, per-span rows/lens,
    codes/gc/flags of span 0) trimmed to nrec."""
    import ctypes

    import torch
    from sctools_amd import _lib
    n = len(data)
    d_buf = torch.tensor(list(data) or [0], dtype=torch.uint8, device="cuda")
    d_ends = torch.tensor(list(ends), dtype=torch.int64, device="cuda")
    cap = max(1, n // 6 + 2) if cap is None else cap
    widths = [e - s for s, e in spans]
    W = sum(widths)
    G = 64  # guard rows past the capacity: nothing may be written there
    seq = torch.full((max(1, (cap + G) * W),), 0xEE, dtype=torch.uint8, device="cuda")
    qual = torch.full_like(seq, 0xEE)
    slen = torch.full((max(1, (cap + G) * len(spans)),), -9, dtype=torch.int32, device="cuda")
    qlen = torch.full_like(slen, -9)
    codes = torch.full((cap + G,), -7, dtype=torch.int64, device="cuda")
    gc = torch.full((cap + G,), 0xEE, dtype=torch.uint8, device="cuda")
    fl = torch.full((cap + G,), 0xEE, dtype=torch.uint8, device="cuda")
    status = torch.full((3,), 77, dtype=torch.int64, device="cuda")
    sp = np.ascontiguousarray(np.array(spans, dtype=np.int32).reshape(-1, 2))
    _lib.check(_lib.lib().sct_fastq_extract_fused(
        d_buf.data_ptr(), n, d_ends.data_ptr(), len(ends), int(text_mode), sp.ctypes.data_as(ctypes.c_void_p),
        len(spans), cap, seq.data_ptr(), qual.data_ptr(), slen.data_ptr(), qlen.data_ptr(),
        codes.data_ptr() if encode else None, gc.data_ptr() if encode else None, fl.data_ptr() if encode else None,
        kind, status.data_ptr(), None))
    torch.cuda.synchronize()
    st = status.cpu().numpy().view(np.uint64)
    nrec = int(st[0]) // 4
    bad = int(~st[1] & np.uint64(0xFFFFFFFFFFFFFFFF)) if int(st[1]) else -1  # raw: no trimming here
    for buf_, fill in ((seq[cap * W:], 0xEE), (qual[cap * W:], 0xEE), (slen[cap * len(spans):], -9),
                       (qlen[cap * len(spans):], -9), (codes[cap:], -7), (gc[cap:], 0xEE), (fl[cap:], 0xEE)):
        assert bool((buf_ == fill).all()), "a row at or past the capacity was written"
    out, off = [], 0
    s_h, q_h = seq.cpu().numpy(), qual.cpu().numpy()
    sl_h, ql_h = slen.cpu().numpy(), qlen.cpu().numpy()
    for k, w in enumerate(widths):
        out.append((s_h[off * cap:(off + w) * cap].reshape(cap, w)[:nrec] if w else np.zeros((nrec, 0), np.uint8),
                    sl_h[k * cap:k * cap + nrec], q_h[off * cap:(off + w) * cap].reshape(cap, w)[:nrec]
                    if w else np.zeros((nrec, 0), np.uint8), ql_h[k * cap:k * cap + nrec]))
        off += w
    enc = (codes.cpu().numpy().view(np.uint64)[:nrec], gc.cpu().numpy()[:nrec], fl.cpu().numpy()[:nrec])
    return nrec, bad, out, enc, int(st[2])


def _fused_cases(fq_golden, tmp_path):
    for case in fq_golden["cases"]:
        blobs = [open(p, "rb").read() for p in _paths(case, tmp_path)]
        yield case["name"], b"".join(blobs), list(np.cumsum([len(b) for b in blobs]))
    rng = np.random.default_rng(8)
    recs = []
    for r in range(200_000):
        L = int(rng.integers(10, 40)) if r % 13 else int(rng.integers(0, 6))  # short reads too
        s = bytes(rng.choice(list(b"ACGTN"), L).tolist())
        q = bytes(rng.integers(33, 75, L).astype(np.uint8).tolist())
        name = b"@r%d" % r if r != 123_457 else b"r%d" % r  # one bad name
        eol = b"\r\n" if r % 7 == 0 else b"\n"
        recs.append(name + eol + s + eol + b"+" + eol + q + eol)
    big = b"".join(recs) + b"@tail\nACGT\n"  # an incomplete trailing record
    cut = [len(big) // 3, len(big) // 3 + 1000, len(big)]  # three files, cuts inside records
    yield "synthetic_200k", big, cut


@pytest.mark.gpu
@pytest.mark.parametrize("text_mode", [0, 1])
def test_fastq_fused_vs_indexed(fq_golden, tmp_path, text_mode):
    """sct_fastq_extract_fused (no index, no scan launch, no host synchronisation; VERDICT r3
    #6) against the indexed two-pass path (itself pinned to the reference's golden outputs
    above): record count, first bad name (the raw status word), every span's sequence / quality
    rows and lengths, and the in-kernel TwoBit and ThreeBit encodes of span 0's rows against
    sct_encode of the same rows."""
    _fused_check(fq_golden, tmp_path, text_mode)


@pytest.mark.gpu
def test_fastq_fused_row_layouts(fq_golden, tmp_path):
    """The fused extraction with slices of widths 9 / 8 / 12 / 33 (rows stored in 1-, 2-, 4- and
    8-byte pieces, a slice of three 16-byte windows, a 9-base encode), against the indexed path."""
    _fused_check(fq_golden, tmp_path, 0, FUSED_SPANS[1])


# TenXV2's CB / UMI (16 + 10) and a 6-wide slice; then widths 9 / 8 / 12 / 33 (rows written in 1-,
# 2-, 4- and 8-byte pieces by the row layout, a slice longer than 32 bytes, a 9-base encode whose
# last dword is partial)
FUSED_SPANS = ([(0, 16), (16, 26), (3, 9)], [(1, 10), (0, 8), (2, 14), (0, 33)])


def _fused_check(fq_golden, tmp_path, text_mode, spans=FUSED_SPANS[0]):
    from sctools_amd import _lib
    for name, data, ends in _fused_cases(fq_golden, tmp_path):
        if text_mode and any(b >= 128 for b in data):
            continue
        n0, bad0, ref = _lib.fastq_extract(data, ends, spans, text_mode)
        n1, bad1, got, enc, na = _fused(data, ends, spans, text_mode)
        assert (n1, bad1, na) == (n0, bad0, 0), name
        for k in range(len(spans)):
            for a, b in zip(ref[k], got[k]):
                assert np.array_equal(np.asarray(a), np.asarray(b)), (name, k)
        if n0:
            w0 = spans[0][1] - spans[0][0]
            codes, gc, flags = _lib.encode(2, np.ascontiguousarray(ref[0][0]), w0)
            assert np.array_equal(enc[0], codes[:, 0]) and np.array_equal(enc[1], gc), name
            assert np.array_equal(enc[2], flags), name
            # ThreeBit (N kept as 6): the queries of the nearest-whitelist correction
            _, _, _, enc3, _ = _fused(data, ends, spans, text_mode, kind=3)
            codes3, gc3, flags3 = _lib.encode(3, np.ascontiguousarray(ref[0][0]), w0)
            assert np.array_equal(enc3[0], codes3[:, 0]) and np.array_equal(enc3[1], gc3), name
            assert np.array_equal(enc3[2], flags3), name
        # a capacity below the record count: the rows below it are the same
        if n0 > 3:
            n2, _, got2, _, _ = _fused(data, ends, spans, text_mode, cap=n0 - 2)
            assert n2 == n0 and np.array_equal(got2[0][0][:n0 - 2], np.asarray(ref[0][0])[:n0 - 2])
