"""Generate tests/golden/fastq_golden.json from the REFERENCE's fastq.EmbeddedBarcodeGenerator.

Runs only in the build container (the reference is at /root/reference), through the same
loader shim as gen_golden.py (stub ``sctools`` package; ``fastq.py`` needs only
``reader.py``).  Inputs are the reference's own test FASTQs (copied here as data
fixtures: tests/golden/fastq/test_r1.fastq, test_i7.fastq) plus small synthetic edge
cases written by this script; outputs are what the reference yields for them, per mode.

Usage:  python tests/golden/gen_fastq_golden.py
"""

import importlib
import json
import os
import sys
import tempfile
import types

REF = "/root/reference/src/sctools"
HERE = os.path.dirname(os.path.abspath(__file__))
FQ = os.path.join(HERE, "fastq")

# edge cases (name -> list of file contents, read in order as one Reader)
EDGE = {
    "short_reads": [b"@r1\nACGTACGTAC\n+\nFFFFFFFFFF\n@r2\nACG\n+\nFFF\n@r3\n\n+\n\n"],
    "no_final_newline": [b"@r1\nACGTACGTACGTACGTAAAACCCCGG\n+\nAAFFJJJJJJJJJJJJJJJJJJJJJJ\n"
                         b"@r2\nTTTTACGTACGTACGTAAAACCCCGG\n+\nAAFFJJJJJJJJJJJJJJJJJJJJJJ"],
    "crlf": [b"@r1\r\nACGTACGTACGTACGTAAAACCCCGG\r\n+\r\nAAFFJJJJJJJJJJJJJJJJJJJJJJ\r\n"],
    "incomplete_record": [b"@r1\nACGTACGTACGTACGTAAAACCCCGG\n+\nAAFFJJJJJJJJJJJJJJJJJJJJJJ\n@r2\nACGT\n"],
    "bad_name": [b"@r1\nACGTACGTACGTACGTAAAACCCCGG\n+\nAAFFJJJJJJJJJJJJJJJJJJJJJJ\n"
                 b"r2\nTTTTACGTACGTACGTAAAACCCCGG\n+\nAAFFJJJJJJJJJJJJJJJJJJJJJJ\n"],
    "record_spans_files": [b"@r1\nACGTACGTACGTACGTAAAACCCCGG\n", b"+\nAAFFJJJJJJJJJJJJJJJJJJJJJJ\n"],
    "unterminated_file_then_file": [b"@r1\nACGTACGTACGTACGTAAAACCCCGG\n+\nAAFFJJJJJJJJJJJJJJJJJJJJJJ",
                                    b"@r2\nGGGGACGTACGTACGTAAAACCCCGG\n+\nAAFFJJJJJJJJJJJJJJJJJJJJJJ\n"],
    "lowercase_and_n": [b"@r1\nacgtNNNNacgtRYKMaaaaccccgg\n+\nAAFFJJJJJJJJJJJJJJJJJJJJJJ\n"],
}

# TenXV2 (platform.py:36-38): (start, end, sequence_tag, quality_tag)
TAGS = {"cell": (0, 16, "CR", "CY"), "molecule": (16, 24, "UR", "UY"), "sample": (0, 8, "SR", "SY")}


def load_reference():
    if not os.path.isdir(REF):
        raise SystemExit("reference not present at %s" % REF)
    pkg = types.ModuleType("sctools")
    pkg.__path__ = [REF]
    sys.modules["sctools"] = pkg
    return importlib.import_module("sctools.fastq")


def enc(x):
    return x.hex() if isinstance(x, bytes) else {"str": x}


def run(fastq, paths, tags, mode):
    ebs = [fastq.EmbeddedBarcode(start=s, end=e, sequence_tag=st, quality_tag=qt)
           for s, e, st, qt in (TAGS[t] for t in tags)]
    out = {"records": []}
    try:
        for rec in fastq.EmbeddedBarcodeGenerator(ebs, paths, mode=mode):
            out["records"].append([[t, enc(v), z] for t, v, z in rec])
    except Exception as e:
        out["error"] = {"type": type(e).__name__, "args": [str(a) for a in e.args]}
    return out


def main():
    fastq = load_reference()
    cases = []
    for files, tags in ((["test_r1.fastq"], ["cell", "molecule"]), (["test_i7.fastq"], ["sample"]),
                        (["test_r1.fastq", "test_r1.fastq"], ["cell"])):
        for mode in ("r", "rb"):
            rec = run(fastq, [os.path.join(FQ, f) for f in files], tags, mode)
            cases.append({"name": "+".join(files), "files": files, "tags": tags, "mode": mode, **rec})
    tmp = tempfile.mkdtemp()
    for name, contents in EDGE.items():
        paths = []
        for k, c in enumerate(contents):
            p = os.path.join(tmp, "%s_%d.fastq" % (name, k))
            with open(p, "wb") as f:
                f.write(c)
            paths.append(p)
        for mode in ("r", "rb"):
            rec = run(fastq, paths, ["cell", "molecule"], mode)
            cases.append({"name": name, "contents": [c.hex() for c in contents], "tags": ["cell", "molecule"],
                          "mode": mode, **rec})
    with open(os.path.join(HERE, "fastq_golden.json"), "w") as f:
        json.dump({"tags": TAGS, "cases": cases}, f)
    print("wrote %d cases" % len(cases))


if __name__ == "__main__":
    main()
