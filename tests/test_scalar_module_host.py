"""The scalar methods' CPython entry points (sctools_amd/csrc/pyscalar.c) on the CPU: the module
is built and importable, and every argument outside the common case returns NotImplemented before
any library call (so the Python methods take their general path, which keeps the reference's
errors).  No call here reaches the GPU."""
import numpy as np

from sctools_amd import _scalar


def test_module_exports():
    for name in ("bind", "hamming", "gc", "decode2", "decode3", "encode"):
        assert callable(getattr(_scalar, name))


def test_uncommon_arguments_are_left_to_python():
    NI = NotImplemented
    assert _scalar.hamming(2, -1, 3) is NI and _scalar.hamming(2, 1 << 64, 0) is NI
    assert _scalar.hamming(2, np.uint64(3), 1) is NI and _scalar.hamming(2, 1.0, 1) is NI
    assert _scalar.hamming(2, 1) is NI  # wrong arity: the Python path raises the TypeError
    assert _scalar.gc(2, -5, 8) is NI and _scalar.gc(2, 5, 0) is NI and _scalar.gc(2, "5", 8) is NI
    assert _scalar.decode2(5, 0) is NI and _scalar.decode2(5, 65) is NI and _scalar.decode2(-5, 4) is NI
    assert _scalar.decode3(-1) is NI and _scalar.decode3(1 << 64) is NI
    for seq in ("ACGT", bytearray(b"ACGT"), memoryview(b"ACGT"), b"", b"A" * 33):
        assert _scalar.encode(2, seq) is NI
    assert _scalar.encode(3, b"A" * 22) is NI and _scalar.encode(4, b"ACGT") is NI
