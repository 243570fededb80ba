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
