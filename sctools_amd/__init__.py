"""sctools_amd — MI355X-native (gfx950) drop-in for sctools' barcode hot path.

``sctools_amd.encodings`` and ``sctools_amd.barcode`` mirror ``sctools.encodings`` and
``sctools.barcode`` (dpeerlab/sctools): TwoBit/ThreeBit encode/decode/gc_content/
hamming_distance and Barcodes (+ ObservedBarcodeSet / PriorBarcodeSet) with the
all-pairs Hamming summary.  Compute runs in HIP kernels of ``libsctools_hip.so``
(C ABI: include/sctools_hip.h) reached through ctypes; nothing falls back to CPU.
Unlike the reference's ``__init__`` this package does not import pysam.
"""

from . import encodings, barcode, stats  # noqa: F401

__version__ = "0.1.0"
