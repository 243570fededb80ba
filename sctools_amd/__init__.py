"""sctools_amd — MI355X-native (gfx950) drop-in for sctools' barcode hot path.

``sctools_amd.encodings`` and ``sctools_amd.barcode`` mirror ``sctools.encodings`` and
``sctools.barcode`` (dpeerlab/sctools): TwoBit/ThreeBit encode/decode/gc_content/
hamming_distance and Barcodes (+ ObservedBarcodeSet / PriorBarcodeSet) with the
all-pairs Hamming summary.  Compute runs in HIP kernels of ``libsctools_hip.so``
(C ABI: include/sctools_hip.h) reached through ctypes; nothing falls back to CPU.
Unlike the reference's ``__init__`` this package does not import pysam.
"""

from . import encodings, barcode, stats  # noqa: F401


def release_device_memory():
    """Free the device workspace that all-pairs summaries keep cached between calls.

    ``Barcodes.summarize_hamming_distances`` on a large set (SPECTRAL) keeps its
    per-device workspace -- up to 4 GiB of transform intermediate -- so the next call maps nothing.
    A process that shares the GPU with another framework can hand that memory back here; the next
    summary call allocates it again (process exit frees it as well).  The idle page-locked host
    blocks the streaming paths keep for their next arrays (``_lib.pinned``) are freed too."""
    from . import _lib
    if _lib._lib is not None:  # nothing to free before the library was loaded
        _lib.release_plan_cache()
        _lib.pinned.trim()


def set_devices(devices):
    """GPUs the drop-in's large calls split over inside the library (the all-pairs summary,
    nearest-whitelist correction, the host encode stream): HIP ordinals, a repeated ordinal being
    a logical shard of one GPU; ``None`` (the default) = every visible device."""
    from . import _lib
    _lib.set_devices(devices)


def keep_workspace(keep=None):
    """False (default): a one-shot all-pairs summary frees all the device memory it mapped before it
    returns.  True: it stays cached per device for the next call (``release_device_memory()``
    hands it back).  Returns the previous setting; ``None`` only reads it."""
    from . import _lib
    return _lib.keep_workspace(keep)


__version__ = "0.1.0"
