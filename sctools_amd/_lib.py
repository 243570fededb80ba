"""ctypes binding of libsctools_hip.so (C ABI declared in include/sctools_hip.h).

This is the only route from the Python drop-in to the hardware: every compute call
of ``sctools_amd.encodings`` / ``sctools_amd.barcode`` lands here and then in a HIP
kernel.  There is no CPU fallback: if the shared library is missing the import of
this module's ``lib()`` raises, and HIP failures (no device, launch errors) surface
as ``RuntimeError`` with the library's message.
"""

import collections
import ctypes
import os
import threading
import weakref

import numpy as np

from . import _scalar

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SCTOOLS_HIP_LIB") or os.path.join(_HERE, "libsctools_hip.so")

SCT_OK = 0
SCT_E_INVALID = -1
SCT_E_HIP = -2
SCT_E_NOMEM = -3
SCT_E_RANGE = -4

# all-pairs count schemes (include/sctools_hip.h)
SCHEME_AUTO = -1
SCHEME_SUBSETS = 0
SCHEME_MOMENTS = 1
SCHEME_SPECTRAL = 2

# launch-shape knobs (sct_tune_set; none changes a result)
TUNE_KEYS = {"spectral_chunk": 1, "spectral_min_n": 2, "allpairs_grab": 3, "allpairs_flush_items": 4,
             "allpairs_grid": 5, "nearest_scheme": 6, "nearest_load": 7, "scalar_server": 8,
             "scalar_idle_ms": 9, "spectral_columns": 10, "plan_cache": 11,
             "encode_grid": 12, "ingest_tiles": 13, "fastq_onepass": 14,
             "ingest_direct": 15, "ingest_spec": 16}
NEAREST_AUTO, NEAREST_OA, NEAREST_CSR, NEAREST_HALVES = 0, 1, 2, 3

_i32, _i64, _dbl = ctypes.c_int, ctypes.c_int64, ctypes.c_double
_vp = ctypes.c_void_p
_p64 = ctypes.POINTER(ctypes.c_uint64)

# name -> argtypes (restype is int unless listed in _RESTYPES); mirrors include/sctools_hip.h
SIGNATURES = {
    "sct_version": [],
    "sct_last_error": [],
    "sct_device_count": [ctypes.POINTER(_i32)],
    "sct_set_device": [_i32],
    "sct_tune_set": [_i32, _i64],
    "sct_tune_get": [_i32, ctypes.POINTER(_i64)],
    "sct_encode": [_i32, _vp, _i64, _i64, _i32, _vp, _vp, _vp, _vp],
    "sct_encode_host": [_i32, _vp, _i64, _i64, _i32, _vp, _vp, _vp],
    "sct_encode_stream_host": [_i32, _vp, _i64, _i32, _vp, _vp, _vp, _i64],
    "sct_host_pinned": [_vp, _i64, _vp],
    "sct_fastq_stream_stage": [_vp, _vp, _i64],
    "sct_nearest_plan_create_host": [_i32, _vp, _i64, _i32, _i32, _vp],
    "sct_nearest_query_host": [_vp, _vp, _i64, _vp, _vp],
    "sct_host_alloc": [_i64, _vp],
    "sct_host_free": [_vp],
    "sct_encode_var": [_i32, _vp, _vp, _vp, _i64, _i32, _vp, _vp, _vp, _vp],
    "sct_lines": [_vp, _i64, _i64, _vp, _vp, ctypes.POINTER(_i64), ctypes.POINTER(_i32), _vp],
    "sct_whitelist_encode": [_vp, _i64, _i32, _i32, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "sct_whitelist_encode_host": [_vp, _i64, _i32, _i32, _i64, ctypes.POINTER(_i64), ctypes.POINTER(_i32), _vp,
                                  _vp, _vp, _vp],
    "sct_decode2": [_vp, _i64, _i32, _i32, _vp, _vp],
    "sct_decode2_host": [_vp, _i64, _i32, _i32, _vp],
    "sct_decode3": [_vp, _i64, _i32, _i32, _vp, _vp, _vp, _vp],
    "sct_decode3_host": [_vp, _i64, _i32, _i32, _vp, _vp, _vp],
    "sct_gc_content": [_i32, _vp, _i64, _i32, _i32, _vp, _vp],
    "sct_gc_content_host": [_i32, _vp, _i64, _i32, _i32, _vp],
    "sct_hamming_pairs": [_i32, _vp, _vp, _i64, _i32, _vp, _vp],
    "sct_hamming_pairs_host": [_i32, _vp, _vp, _i64, _i32, _vp],
    "sct_allpairs_plan_create": [_vp, _i64, _i32, ctypes.POINTER(_vp)],
    "sct_allpairs_plan_create_ex": [_vp, _i64, _i32, _i32, ctypes.POINTER(_vp)],
    "sct_allpairs_plan_scheme": [_vp, ctypes.POINTER(_i32), ctypes.POINTER(_i32), ctypes.POINTER(_i32)],
    "sct_allpairs_moments": [_vp, _i32, _i32, _vp, _vp],
    "sct_allpairs_plan_destroy": [_vp],
    "sct_allpairs_plan_info": [_vp, ctypes.POINTER(_i32), ctypes.POINTER(_i64), ctypes.POINTER(_i64)],
    "sct_allpairs_build": [_vp, _vp],
    "sct_allpairs_build_items": [_vp, _i64, _i64, _vp],
    "sct_allpairs_count": [_vp, _i64, _i64, _vp, _i32, _vp],
    "sct_allpairs_range_pairs": [_vp, _i64, _i64, ctypes.POINTER(_i64)],
    "sct_allpairs_time_kernels": [_vp, _i64, _i64, _vp, _i32, ctypes.POINTER(ctypes.c_double), _vp],
    "sct_allpairs_timing": [_vp, _i32, ctypes.POINTER(ctypes.c_double)],
    "sct_allpairs_spectral_info": [_vp, ctypes.POINTER(_i32), ctypes.POINTER(_i64), ctypes.POINTER(_i32)],
    "sct_allpairs_spectral_columns": [_vp, ctypes.POINTER(_i32)],
    "sct_nearest_plan_info": [_vp, ctypes.POINTER(_i32), ctypes.POINTER(_i64)],
    "sct_allpairs_geometry": [_i64, _i32, ctypes.POINTER(_i32), ctypes.POINTER(_i64),
                              ctypes.POINTER(_i32), ctypes.POINTER(_i32)],
    "sct_counts_to_hist": [_vp, _i32, _vp],
    "sct_counts_to_hist_ex": [_i32, _vp, _i32, _vp, _i32],
    "sct_hamming_hist_allpairs_host": [_vp, _i64, _i32, _vp, _i32],
    "sct_hamming_hist_allpairs_host_ex": [_vp, _i64, _i32, _i32, _vp, _i32],
    "sct_allpairs_plan_create_ex2": [_vp, _i64, _i32, _i32, _i32, ctypes.POINTER(_vp)],
    "sct_allpairs_cache_release": [],
    "sct_summary_from_hist": [_vp, _i32, _vp],
    "sct_allpairs_wide_geometry": [_i64, _i32, ctypes.POINTER(_i64), ctypes.POINTER(_i32)],
    "sct_allpairs_wide_range_pairs": [_i64, _i64, _i64, ctypes.POINTER(_i64)],
    "sct_allpairs_wide": [_vp, _i64, _i32, _i64, _i64, _vp, _i32, _vp],
    "sct_hamming_hist_allpairs_wide_host": [_vp, _i64, _i32, _vp, _i32],
    "sct_nearest_plan_create": [_i32, _vp, _i64, _i32, _i32, _vp, ctypes.POINTER(_vp)],
    "sct_nearest_plan_destroy": [_vp],
    "sct_nearest_query": [_vp, _vp, _i64, _vp, _vp, _vp],
    "sct_nearest_host": [_i32, _vp, _i64, _vp, _i64, _i32, _i32, _vp, _vp],
    "sct_base_frequency": [_vp, _i64, _i32, _vp, _vp],
    "sct_fastq_index_create": [_vp, _i64, _vp, _i32, _i32, _vp, ctypes.POINTER(_vp)],
    "sct_fastq_index_destroy": [_vp],
    "sct_fastq_index_info": [_vp, ctypes.POINTER(_i64), ctypes.POINTER(_i64), ctypes.POINTER(_i64)],
    "sct_fastq_extract_spans": [_vp, _vp, _vp, _i32, _vp, _vp, _vp, _vp, ctypes.POINTER(_i64), _vp],
    "sct_fastq_extract_host": [_vp, _i64, _vp, _i32, _i32, _vp, _i32, _vp, _vp, _vp, _vp, _i64,
                               ctypes.POINTER(_i64), ctypes.POINTER(_i64)],
    "sct_base_frequency_host": [_vp, _i64, _i32, _vp],
    "sct_fastq_extract_fused": [_vp, _i64, _vp, _i32, _i32, _vp, _i32, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                _i32, _vp, _vp],
    "sct_fastq_stream_create": [_i32, _vp, _i32, _i32, ctypes.POINTER(_vp)],
    "sct_fastq_stream_destroy": [_vp],
    "sct_fastq_stream_chunk": [_vp, _vp, _i64, _vp, _i32, _i32, ctypes.POINTER(_i64), ctypes.POINTER(_i64),
                               ctypes.POINTER(_i64)],
    "sct_fastq_stream_fetch": [_vp, _vp, _vp, _vp, _vp],
    "sct_scalar_server_stop": [],
    "sct_stream_copy": [_vp, _vp, _i64, _vp],
    "sct_scalar_server_status": [ctypes.POINTER(_i64), ctypes.POINTER(_i32)],
    "sct_keep_workspace": [_i32, ctypes.POINTER(_i32)],
    "sct_hamming_hist_allpairs_host_devices": [_vp, _i64, _i32, _i32, _vp, _i32, _vp, _i32],
    "sct_nearest_host_devices": [_i32, _vp, _i64, _vp, _i64, _i32, _i32, _vp, _i32, _vp, _vp],
    "sct_nearest_multi_create_host": [_i32, _vp, _i64, _i32, _i32, _vp, _i32, ctypes.POINTER(_vp)],
    "sct_nearest_multi_query_host": [_vp, _vp, _i64, _vp, _vp],
    "sct_nearest_multi_destroy": [_vp],
    "sct_encode_stream_host_devices": [_i32, _vp, _i64, _i32, _vp, _vp, _vp, _i64, _vp, _i32],
}
_RESTYPES = {"sct_last_error": ctypes.c_char_p}

_lock = threading.Lock()
_lib = None


class LibraryMissing(ImportError):
    pass


def _torch_hip_runtime():
    """Path of the HIP runtime bundled with torch (found without importing torch)."""
    try:
        import importlib.util
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        return None
    if spec is None or not spec.submodule_search_locations:
        return None
    path = os.path.join(list(spec.submodule_search_locations)[0], "lib", "libamdhip64.so")
    return path if os.path.exists(path) else None


def lib():
    """Load libsctools_hip.so once; raise LibraryMissing (an ImportError) if absent.

    torch ships its own libamdhip64 with the same SONAME (libamdhip64.so.7) as ROCm's;
    two HIP runtimes in one process break each other ("No HIP GPUs are available").
    So when torch is installed its runtime is loaded first (RTLD_GLOBAL) and this
    library binds to it, whatever the import order."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise LibraryMissing(
                    "libsctools_hip.so not found at %s: build it with "
                    "`python -c 'import __graft_entry__; __graft_entry__.build()'` "
                    "(there is no CPU fallback)" % LIB_PATH)
            rt = os.environ.get("SCTOOLS_HIP_RUNTIME") or _torch_hip_runtime()
            if rt:
                ctypes.CDLL(rt, mode=ctypes.RTLD_GLOBAL)
            handle = ctypes.CDLL(LIB_PATH)
            for name, args in SIGNATURES.items():
                fn = getattr(handle, name)
                fn.argtypes = args
                fn.restype = _RESTYPES.get(name, _i32)
            # the scalar methods' CPython entry points call these directly (csrc/pyscalar.c)
            _scalar.bind(*(ctypes.cast(getattr(handle, name), ctypes.c_void_p).value
                           for name in ("sct_hamming_pairs_host", "sct_gc_content_host", "sct_decode2_host",
                                        "sct_encode_host", "sct_decode3_host")))
            _lib = handle
    return _lib


def last_error():
    msg = lib().sct_last_error()
    return msg.decode("utf-8", "replace") if msg else ""


def check(rc):
    if rc == SCT_OK:
        return
    msg = last_error()
    if rc == SCT_E_NOMEM:
        raise MemoryError(msg)
    if rc in (SCT_E_INVALID, SCT_E_RANGE):
        raise ValueError(msg)
    raise RuntimeError(msg)


def tune_get(name):
    v = _i64(0)
    check(lib().sct_tune_get(TUNE_KEYS[name], ctypes.byref(v)))
    return v.value


def tune_set(name, value):
    """Set a launch-shape knob (None or < 0 restores the default)."""
    check(lib().sct_tune_set(TUNE_KEYS[name], -1 if value is None else int(value)))


class tuning:
    """Context manager: ``with tuning(spectral_chunk=1000): ...`` sets knobs and restores them."""

    def __init__(self, **knobs):
        self.knobs = knobs
        self.saved = {}

    def __enter__(self):
        for k, v in self.knobs.items():
            self.saved[k] = tune_get(k)
            tune_set(k, v)
        return self

    def __exit__(self, *exc):
        for k, v in self.saved.items():
            tune_set(k, v)
        return False


def _ptr(a):
    return a.ctypes.data_as(_vp) if a is not None else None


# ------------------------------------------------------------------ devices
# The drop-in's large calls split over these devices inside the library (devices.cpp: one worker
# thread per slot, no torch.distributed): the all-pairs summary from the SPECTRAL threshold, nearest
# and the host encode stream from MULTI_MIN_RECORDS.  None = every visible device.
_devices = None
MULTI_MIN_RECORDS = 1 << 22


def set_devices(devices):
    """Use ``devices`` (HIP ordinals; a repeated ordinal is a logical shard of one GPU) for the
    drop-in's multi-device calls; ``None`` restores the default, every visible device."""
    global _devices
    if devices is None:
        _devices = None
        return
    devs = [int(d) for d in devices]
    if not devs:
        raise ValueError("set_devices needs at least one device")
    _devices = devs


def get_devices():
    """The devices multi-device calls split over (default: every visible device)."""
    if _devices is not None:
        return list(_devices)
    n = device_count()
    return list(range(n)) if n > 1 else [0]


def _devs(devices, size, threshold):
    """The device list a call of ``size`` records uses: the explicit one, else the configured
    devices when the call is large enough to split; None = the current device alone."""
    if devices is not None:
        devs = [int(d) for d in devices]
        return devs if len(devs) > 1 else None
    if size < threshold:
        return None
    devs = get_devices()
    return devs if len(devs) > 1 else None


def _dev_array(devs):
    return (ctypes.c_int * len(devs))(*devs)


def keep_workspace(keep=None):
    """The all-pairs one-shot's device memory policy; returns the previous setting.  False (the
    default): a call frees every device buffer it allocated before it returns (a 737K summary maps
    and unmaps its 4 GiB transform intermediate each time).  True: the buffers stay cached per
    device, so repeated calls map nothing (``release_device_memory()`` frees them).  None: read."""
    prev = _i32(0)
    check(lib().sct_keep_workspace(-1 if keep is None else int(bool(keep)), ctypes.byref(prev)))
    return bool(prev.value)


def _spectral_min_n():
    v = tune_get("spectral_min_n")
    return 325000 if v < 0 else v


# ------------------------------------------------------------------ int <-> limbs
def words_for_bits(bits):
    return max(1, -(-int(bits) // 64))


def ints_to_limbs(values, words=None):
    """Python ints (>= 0) -> (n, words) uint64 little-endian limbs."""
    values = list(values)
    if words is None:
        words = words_for_bits(max((int(v).bit_length() for v in values), default=0))
    if words == 1:
        return np.array(values, dtype=np.uint64).reshape(-1, 1)
    buf = b"".join(int(v).to_bytes(8 * words, "little") for v in values)
    return np.frombuffer(buf, dtype="<u8").reshape(-1, words).astype(np.uint64)


def limbs_to_ints(limbs):
    limbs = np.ascontiguousarray(limbs, dtype=np.uint64)
    if limbs.ndim == 1 or limbs.shape[1] == 1:
        return [int(x) for x in limbs.reshape(-1).tolist()]
    return [int.from_bytes(row.astype("<u8").tobytes(), "little") for row in limbs]


# ------------------------------------------------------------------ scalar calls
# The drop-in's scalar methods (TwoBit.encode(bytes) -> int, ...) are batches of one; these
# helpers pass one-limb values through per-thread ctypes buffers (no numpy arrays per call)
# into the library's zero-copy host stage.
_tls = threading.local()


def _scalar_bufs():
    b = getattr(_tls, "bufs", None)
    if b is None:
        b = _tls.bufs = {"a": (ctypes.c_uint64 * 1)(), "b": (ctypes.c_uint64 * 1)(), "i": (ctypes.c_int32 * 1)(),
                         "gc": (ctypes.c_uint8 * 1)(), "fl": (ctypes.c_uint8 * 1)(), "out": ctypes.create_string_buffer(64)}
    return b


def hamming1(kind, a, b):
    """One pair of one-limb codes (< 2^64) -> distance."""
    bufs = _scalar_bufs()
    bufs["a"][0] = a
    bufs["b"][0] = b
    check(lib().sct_hamming_pairs_host(kind, ctypes.addressof(bufs["a"]), ctypes.addressof(bufs["b"]), 1, 1,
                                       ctypes.addressof(bufs["i"])))
    return bufs["i"][0]


def gc1(kind, code, L=0):
    bufs = _scalar_bufs()
    bufs["a"][0] = code
    check(lib().sct_gc_content_host(kind, ctypes.addressof(bufs["a"]), 1, 1, L, ctypes.addressof(bufs["i"])))
    return bufs["i"][0]


def encode1(kind, seq):
    """One record of L <= 64 / kind bytes -> (code, flags): a one-limb code."""
    bufs = _scalar_bufs()
    L = len(seq)
    check(lib().sct_encode_host(kind, seq, 1, L, L, ctypes.addressof(bufs["a"]), None,
                                ctypes.addressof(bufs["fl"])))
    return bufs["a"][0], bufs["fl"][0]


def decode2_1(code, L):
    """One one-limb TwoBit code -> L bytes (L <= 64)."""
    bufs = _scalar_bufs()
    bufs["a"][0] = code
    out = bufs["out"]
    check(lib().sct_decode2_host(ctypes.addressof(bufs["a"]), 1, 1, L, ctypes.addressof(out)))
    return out.raw[:L]


# ------------------------------------------------------------------ entry points
def encode(kind, seqs, L):
    """(n, L) uint8 array -> (codes (n, words) uint64, gc uint8|None, flags uint8)."""
    seqs = np.ascontiguousarray(seqs, dtype=np.uint8).reshape(-1, L) if L else np.zeros((len(seqs), 0), np.uint8)
    n = seqs.shape[0]
    words = words_for_bits(kind * L)
    codes = np.zeros((n, words), dtype=np.uint64)
    flags = np.zeros(n, dtype=np.uint8)
    gc = np.zeros(n, dtype=np.uint8) if L <= 255 else None
    check(lib().sct_encode_host(kind, _ptr(seqs), n, L, L, _ptr(codes), _ptr(gc), _ptr(flags)))
    return codes, gc, flags


def encode_stream(kind, seqs, chunk=0, devices=None):
    """Host (n, L) uint8 records -> (codes uint64[n], gc uint8[n], flags uint8[n]) through the
    pipelined H2D/encode/D2H stream (one limb per code); large batches split over the devices
    (contiguous record ranges, see set_devices)."""
    seqs = np.ascontiguousarray(seqs, dtype=np.uint8)
    n, L = seqs.shape
    codes = pinned.empty(n, np.uint64)
    gc = pinned.empty(n, np.uint8)
    flags = pinned.empty(n, np.uint8)
    devs = _devs(devices, n, MULTI_MIN_RECORDS)
    if devs:
        check(lib().sct_encode_stream_host_devices(kind, _ptr(seqs), n, L, _ptr(codes), _ptr(gc), _ptr(flags), chunk,
                                                   _dev_array(devs), len(devs)))
    else:
        check(lib().sct_encode_stream_host(kind, _ptr(seqs), n, L, _ptr(codes), _ptr(gc), _ptr(flags), chunk))
    return codes, gc, flags


def host_pinned(arr):
    """True when the numpy array's bytes lie in one page-locked allocation (DMA in place)."""
    out = _i32(0)
    check(lib().sct_host_pinned(_vp(arr.ctypes.data), arr.nbytes, ctypes.byref(out)))
    return bool(out.value)


class PinnedPool:
    """Page-locked host blocks (sct_host_alloc) behind numpy arrays: the host stream paths read
    files into them and copy device results into them, so every PCIe crossing is a DMA in place
    and a reused block takes no page faults.  An array (with every view of it) hands its block
    back when it is freed; up to ``keep_bytes`` of idle blocks stay for the next arrays, the rest
    are freed.  At most ``max_bytes`` are page-locked at a time (default: a quarter of the host's
    memory, at most 16 GiB): past that -- a caller keeping every piece of a long stream -- new
    arrays are plain numpy arrays again.  Small arrays, and every array once page-locked memory
    is refused (no GPU, or the allocation fails), are plain numpy arrays."""

    MIN_BYTES = 1 << 20

    def __init__(self, keep_bytes=2 << 30, max_bytes=None):
        self.keep_bytes = int(keep_bytes)
        if max_bytes is None:
            try:
                phys = os.sysconf("SC_PHYS_PAGES") * os.sysconf("SC_PAGE_SIZE")
            except (ValueError, OSError, AttributeError):
                phys = 64 << 30
            max_bytes = min(16 << 30, phys // 4)
        self.max_bytes = int(max_bytes)
        self._free = {}  # size class -> [pointer]
        self._idle = 0
        self._held = 0  # page-locked bytes: blocks behind live arrays + idle blocks
        self._mu = threading.Lock()
        self._pending = collections.deque()  # blocks handed back, not yet filed under _mu
        self._order = collections.deque()  # idle (size class, pointer) in the order they went idle
        self._ok = True
        self._types = {}

    @staticmethod
    def _class(nbytes):
        c = PinnedPool.MIN_BYTES
        while c < nbytes:
            c <<= 1
        return c

    def empty(self, shape, dtype=np.uint8):
        shape = (shape,) if isinstance(shape, (int, np.integer)) else tuple(shape)
        dtype = np.dtype(dtype)
        count = int(np.prod(shape, dtype=np.int64)) if shape else 1
        nbytes = count * dtype.itemsize
        if nbytes < self.MIN_BYTES or not self._ok:
            return np.empty(shape, dtype)
        c = self._class(nbytes)
        self._drain()
        with self._mu:
            blocks = self._free.get(c)
            ptr = blocks.pop() if blocks else None
            if ptr is not None:
                self._idle -= c
                self._order.remove((c, ptr))
        if ptr is None:
            with self._mu:
                if self._held + c > self.max_bytes:
                    return np.empty(shape, dtype)
                self._held += c
            p = _vp()
            if lib().sct_host_alloc(c, ctypes.byref(p)) != SCT_OK or not p.value:
                with self._mu:
                    self._held -= c
                self._ok = False  # (no GPU, or page-locked memory refused: plain arrays from now on)
                return np.empty(shape, dtype)
            ptr = p.value
        t = self._types.get(c)
        if t is None:
            t = self._types[c] = ctypes.c_uint8 * c
        buf = t.from_address(ptr)
        fin = weakref.finalize(buf, self._release, ptr, c)
        fin.atexit = False  # (at interpreter exit the process returns the memory)
        return np.frombuffer(buf, dtype=dtype, count=count).reshape(shape)

    def _release(self, ptr, c):
        # a weakref.finalize callback: it can run inside a cyclic collection that an allocation
        # made while this thread holds _mu started, so it never waits on _mu -- the
        # block goes on a lock-free queue and whoever holds or next takes the lock files it
        self._pending.append((ptr, c))
        self._drain()

    def _drain(self):
        if not self._mu.acquire(blocking=False):
            return  # (the holder -- maybe this very thread -- drains the queue before it lets go)
        to_free = []
        try:
            while self._pending:
                ptr, c = self._pending.popleft()
                if c > self.keep_bytes:
                    self._held -= c
                    to_free.append(ptr)
                    continue
                # the block just handed back stays; the longest-idle ones make room for it (a
                # stream of equal calls then reuses its blocks instead of page-locking anew)
                while self._idle + c > self.keep_bytes:
                    oc, op = self._order.popleft()
                    self._free[oc].remove(op)
                    self._idle -= oc
                    self._held -= oc
                    to_free.append(op)
                self._free.setdefault(c, []).append(ptr)
                self._order.append((c, ptr))
                self._idle += c
        finally:
            self._mu.release()
        for p in to_free:
            lib().sct_host_free(_vp(p))
        if self._pending:  # (queued by another thread between the last pop and the release)
            self._drain()

    def trim(self):
        """Free every idle block."""
        self._drain()
        with self._mu:
            ptrs = [p for blocks in self._free.values() for p in blocks]
            self._free.clear()
            self._order.clear()
            self._held -= self._idle
            self._idle = 0
        self._drain()  # (blocks handed back while the lock was held go idle, then stay for reuse)
        for p in ptrs:
            lib().sct_host_free(_vp(p))


pinned = PinnedPool()


def whitelist_encode(data, kind=2):
    """Whitelist file bytes -> every line's [:-1] encoded on the device (barcode.py:95-97):
    (codes (n, words) uint64, starts int64[n], chopped lengths int32[n], flags uint8[n])."""
    buf = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
    n, mx = _i64(0), _i32(0)
    f = lib().sct_whitelist_encode_host
    check(f(_ptr(buf), len(data), kind, 1, 0, ctypes.byref(n), ctypes.byref(mx), None, None, None, None))
    nl = n.value
    words = words_for_bits(kind * mx.value)
    codes = np.zeros((nl, words), dtype=np.uint64)
    starts = np.zeros(nl, dtype=np.int64)
    lens = np.zeros(nl, dtype=np.int32)
    flags = np.zeros(nl, dtype=np.uint8)
    if nl:
        check(f(_ptr(buf), len(data), kind, words, nl, ctypes.byref(n), ctypes.byref(mx), _ptr(codes),
                _ptr(starts), _ptr(lens), _ptr(flags)))
    return codes, starts, lens, flags


# Element-wise batch outputs come from the page-locked pool (large calls then DMA their results
# in place: the library streams them in chunks, include/sctools_hip.h); every element is written.
def decode2(codes, L):
    codes = np.ascontiguousarray(codes, dtype=np.uint64)
    codes2 = codes.reshape(codes.shape[0], -1)
    out = pinned.empty((codes2.shape[0], L), np.uint8)
    check(lib().sct_decode2_host(_ptr(codes2), codes2.shape[0], codes2.shape[1], L, _ptr(out)))
    return out


def decode3(codes):
    codes = np.ascontiguousarray(codes, dtype=np.uint64)
    codes2 = codes.reshape(codes.shape[0], -1)
    n, words = codes2.shape
    maxlen = (64 * words + 2) // 3
    out = pinned.empty((n, maxlen), np.uint8)  # (row r's bytes before its right-aligned sequence: unset)
    lengths = pinned.empty(n, np.int32)
    bad = pinned.empty(n, np.int32)
    check(lib().sct_decode3_host(_ptr(codes2), n, words, maxlen, _ptr(out), _ptr(lengths), _ptr(bad)))
    return out, lengths, bad


def gc_content(kind, codes, L=0):
    codes = np.ascontiguousarray(codes, dtype=np.uint64)
    codes2 = codes.reshape(codes.shape[0], -1)
    out = pinned.empty(codes2.shape[0], np.int32)
    check(lib().sct_gc_content_host(kind, _ptr(codes2), codes2.shape[0], codes2.shape[1], L, _ptr(out)))
    return out


def hamming_pairs(kind, a, b):
    a = np.ascontiguousarray(a, dtype=np.uint64)
    b = np.ascontiguousarray(b, dtype=np.uint64)
    a2 = a.reshape(a.shape[0], -1)
    b2 = b.reshape(b.shape[0], -1)
    if a2.shape != b2.shape:
        raise ValueError("operand shapes differ: %s vs %s" % (a2.shape, b2.shape))
    out = pinned.empty(a2.shape[0], np.int32)
    check(lib().sct_hamming_pairs_host(kind, _ptr(a2), _ptr(b2), a2.shape[0], a2.shape[1], _ptr(out)))
    return out


def nbins_for_bits(code_bits):
    return 2 * ((max(1, int(code_bits)) + 3) // 4) + 1


ALLPAIRS_DISTINCT = 1  # plan flag: the caller promises pairwise-distinct codes


def hamming_hist_allpairs(codes, code_bits=None, distinct=False, devices=None):
    """Histogram (uint64[nbins]) of TwoBit distances over all unordered pairs of codes.
    distinct=True promises pairwise-distinct codes (mapping keys): SPECTRAL then skips its
    sort for sum f^2; a broken promise raises ValueError (the host's exact check), never a
    wrong histogram.  devices: the device slots to split over (default: every device of
    set_devices() once the set reaches the SPECTRAL threshold; one device below it)."""
    codes = np.ascontiguousarray(codes, dtype=np.uint64).reshape(-1)
    if code_bits is None:  # bit_length(max) = bit_length(OR) for non-negative codes
        code_bits = int(codes.max()).bit_length() if codes.size else 1
    code_bits = max(1, code_bits)
    nbins = nbins_for_bits(code_bits)
    hist = np.zeros(nbins, dtype=np.uint64)
    flags = ALLPAIRS_DISTINCT if distinct else 0
    devs = _devs(devices, codes.size, _spectral_min_n())
    if devs:
        check(lib().sct_hamming_hist_allpairs_host_devices(_ptr(codes), codes.size, code_bits, flags, _dev_array(devs),
                                                           len(devs), _ptr(hist), nbins))
    else:
        check(lib().sct_hamming_hist_allpairs_host_ex(_ptr(codes), codes.size, code_bits, flags, _ptr(hist), nbins))
    return hist


def release_plan_cache():
    """Free the device buffers all-pairs plans keep cached between calls (sct_allpairs_cache_release)."""
    check(lib().sct_allpairs_cache_release())


def hamming_hist_allpairs_wide(limbs):
    """Histogram (uint64[32*words+1]) of TwoBit distances over all unordered pairs of
    multi-limb codes ((n, words) little-endian uint64: Python ints of any size)."""
    limbs = np.ascontiguousarray(limbs, dtype=np.uint64)
    limbs = limbs.reshape(limbs.shape[0], -1) if limbs.ndim else limbs.reshape(0, 1)
    n, words = limbs.shape
    hist = np.zeros(32 * words + 1, dtype=np.uint64)
    check(lib().sct_hamming_hist_allpairs_wide_host(_ptr(limbs), n, words, _ptr(hist), hist.size))
    return hist


def wide_geometry(n, words):
    """(items, nbins) of the wide all-pairs kernel (host arithmetic)."""
    it, nb = _i64(0), _i32(0)
    check(lib().sct_allpairs_wide_geometry(n, words, ctypes.byref(it), ctypes.byref(nb)))
    return it.value, nb.value


def wide_range_pairs(n, begin, end):
    p = _i64(0)
    check(lib().sct_allpairs_wide_range_pairs(n, begin, end, ctypes.byref(p)))
    return p.value


def counts_to_hist(counts, scheme=SCHEME_SUBSETS, nbins=None):
    """Counts of an all-pairs plan (any scheme) -> exact histogram (uint64[nbins])."""
    counts = np.ascontiguousarray(counts, dtype=np.uint64).reshape(-1)
    if nbins is None:  # SPECTRAL counts: n, sum f^2 and three limbs of the 17 weight sums
        nbins = 17 if scheme == SCHEME_SPECTRAL else counts.size
    hist = np.zeros(nbins, dtype=np.uint64)
    check(lib().sct_counts_to_hist_ex(scheme, _ptr(counts), counts.size, _ptr(hist), nbins))
    return hist


def summary_from_hist(hist):
    """6 float64: minimum, 25th, median, 75th percentile, maximum, average (bit-exact numpy)."""
    hist = np.ascontiguousarray(hist, dtype=np.uint64).reshape(-1)
    out = np.zeros(6, dtype=np.float64)
    rc = lib().sct_summary_from_hist(_ptr(hist), hist.size, _ptr(out))
    if rc == SCT_E_RANGE and int(hist.sum()) == 0:
        # np.percentile of an empty list (barcode.py:45 with < 2 unique barcodes)
        raise IndexError("index -1 is out of bounds for axis 0 with size 0")
    check(rc)
    return out


def base_frequency(codes, L):
    codes = np.ascontiguousarray(codes, dtype=np.uint64).reshape(-1)
    out = np.zeros((L, 4), dtype=np.uint64)
    check(lib().sct_base_frequency_host(_ptr(codes), codes.size, L, _ptr(out)))
    return out


def fastq_extract(buf, file_ends, spans, text_mode, qualities=True):
    """Device FASTQ slicing.  buf: bytes of the concatenated files; file_ends: cumulative
    ends; spans: [(start, end)].  Returns (nrecords, first_bad_name, [(seq (n, w) uint8,
    seq_len int32[n], qual (n, w) uint8 | None, qual_len | None) per span])."""
    data = np.frombuffer(buf, dtype=np.uint8) if len(buf) else np.zeros(1, np.uint8)
    ends = np.ascontiguousarray(file_ends, dtype=np.int64)
    sp = np.ascontiguousarray(np.array(spans, dtype=np.int32).reshape(-1, 2))
    nrec, bad = _i64(0), _i64(0)
    f = lib().sct_fastq_extract_host
    check(f(_ptr(data), len(buf), _ptr(ends), ends.size, int(text_mode), _ptr(sp), sp.shape[0],
            None, None, None, None, -1, ctypes.byref(nrec), ctypes.byref(bad)))
    n = nrec.value
    widths = [int(e - s) for s, e in sp]
    seq = np.zeros(max(1, n * sum(widths)), dtype=np.uint8)
    qual = np.zeros_like(seq) if qualities else None
    slen = np.zeros(max(1, n * len(widths)), dtype=np.int32)
    qlen = np.zeros_like(slen) if qualities else None
    check(f(_ptr(data), len(buf), _ptr(ends), ends.size, int(text_mode), _ptr(sp), sp.shape[0],
            _ptr(seq), _ptr(qual), _ptr(slen), _ptr(qlen), n, ctypes.byref(nrec), ctypes.byref(bad)))
    out, off = [], 0
    for k, w in enumerate(widths):
        rows = seq[off:off + n * w].reshape(n, w)
        q = qual[off:off + n * w].reshape(n, w) if qualities else None
        out.append((rows, slen[k * n:(k + 1) * n], q, qlen[k * n:(k + 1) * n] if qualities else None))
        off += n * w
    return n, bad.value, out


class FastqStream:
    """Chunked FASTQ extraction (sct_fastq_stream): device buffers kept across pieces."""

    def __init__(self, spans, text_mode, qualities=True):
        self._lib = lib()
        self._h = _vp()
        self.spans = [(int(a), int(b)) for a, b in spans]
        self.qualities = bool(qualities)
        sp = np.ascontiguousarray(np.array(self.spans, dtype=np.int32).reshape(-1, 2))
        check(self._lib.sct_fastq_stream_create(int(text_mode), _ptr(sp), sp.shape[0], int(qualities),
                                                ctypes.byref(self._h)))

    def chunk(self, buf, nbytes, file_ends, final):
        """Extract the complete records of buf[:nbytes] (a writable or read-only buffer);
        returns (nrecords, consumed, first_bad, [(seq, seq_len, qual, qual_len) per span])."""
        data = np.frombuffer(buf, dtype=np.uint8, count=nbytes) if nbytes else np.zeros(1, np.uint8)
        ends = np.ascontiguousarray(file_ends, dtype=np.int64)
        n, used, bad = _i64(0), _i64(0), _i64(0)
        check(self._lib.sct_fastq_stream_chunk(self._h, _ptr(data), nbytes, _ptr(ends), ends.size, int(final),
                                               ctypes.byref(n), ctypes.byref(used), ctypes.byref(bad)))
        del data
        nr = n.value
        widths = [b - a for a, b in self.spans]
        # (the fetch fills every element; page-locked rows come back by DMA in place)
        seq = pinned.empty(max(1, nr * sum(widths)), np.uint8)
        qual = pinned.empty(seq.size, np.uint8) if self.qualities else None
        slen = pinned.empty(max(1, nr * len(widths)), np.int32)
        qlen = pinned.empty(slen.size, np.int32) if self.qualities else None
        check(self._lib.sct_fastq_stream_fetch(self._h, _ptr(seq), _ptr(qual), _ptr(slen), _ptr(qlen)))
        out, off = [], 0
        for k, w in enumerate(widths):
            rows = seq[off:off + nr * w].reshape(nr, w)
            q = qual[off:off + nr * w].reshape(nr, w) if self.qualities else None
            out.append((rows, slen[k * nr:(k + 1) * nr], q, qlen[k * nr:(k + 1) * nr] if self.qualities else None))
            off += nr * w
        return nr, used.value, bad.value, out

    def stage(self, buf, nbytes):
        """Copy the next piece buf[:nbytes] to the device now (page-locked buffers only); the
        chunk call for the same buffer and size then skips its copy.  buf must stay unchanged
        until that call."""
        data = np.frombuffer(buf, dtype=np.uint8, count=nbytes) if nbytes else np.zeros(1, np.uint8)
        check(self._lib.sct_fastq_stream_stage(self._h, _ptr(data), nbytes))

    def close(self):
        if self._h:
            self._lib.sct_fastq_stream_destroy(self._h)
            self._h = _vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class FastqIndex:
    """Device FASTQ line/record index over a device buffer (sct_fastq_index)."""

    def __init__(self, d_buf_ptr, nbytes, file_ends, text_mode=False, stream=0):
        self._lib = lib()
        self._h = _vp()
        ends = np.ascontiguousarray(file_ends, dtype=np.int64)
        check(self._lib.sct_fastq_index_create(_vp(d_buf_ptr), nbytes, _ptr(ends), ends.size,
                                               int(text_mode), _vp(stream), ctypes.byref(self._h)))
        nr, nl, bad = _i64(0), _i64(0), _i64(0)
        check(self._lib.sct_fastq_index_info(self._h, ctypes.byref(nr), ctypes.byref(nl), ctypes.byref(bad)))
        self.nrecords, self.nlines, self.first_bad_name = nr.value, nl.value, bad.value

    def extract_spans(self, d_buf_ptr, spans, d_seq_ptr, d_qual_ptr=0, d_seq_len_ptr=0,
                      d_qual_len_ptr=0, stream=0):
        """All spans of every record in one pass; returns the first bad-name record or -1."""
        sp = np.ascontiguousarray(np.array(spans, dtype=np.int32).reshape(-1, 2))
        bad = _i64(0)
        check(self._lib.sct_fastq_extract_spans(self._h, _vp(d_buf_ptr), _ptr(sp), sp.shape[0],
                                                _vp(d_seq_ptr), _vp(d_qual_ptr), _vp(d_seq_len_ptr),
                                                _vp(d_qual_len_ptr), ctypes.byref(bad), _vp(stream)))
        self.first_bad_name = bad.value
        return bad.value

    def close(self):
        if self._h:
            self._lib.sct_fastq_index_destroy(self._h)
            self._h = _vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def allpairs_geometry(n, code_bits):
    """Host-only plan geometry: dict(nbins, items, rows_per_item, cols_per_item)."""
    nb, it, rb, cb = _i32(0), _i64(0), _i32(0), _i32(0)
    check(lib().sct_allpairs_geometry(n, code_bits, ctypes.byref(nb), ctypes.byref(it),
                                      ctypes.byref(rb), ctypes.byref(cb)))
    return {"nbins": nb.value, "items": it.value, "rows_per_item": rb.value, "cols_per_item": cb.value}


def nearest(kind, whitelist, queries, max_d=1, code_bits=None, devices=None):
    """Brute-force-equivalent nearest whitelist entry -> (index int32, dist uint8); large query
    sets split over the devices (contiguous ranges, the whitelist indexed on each)."""
    wl = np.ascontiguousarray(whitelist, dtype=np.uint64).reshape(-1)
    q = np.ascontiguousarray(queries, dtype=np.uint64).reshape(-1)
    if code_bits is None:
        code_bits = max(1, int(np.bitwise_or.reduce(wl)).bit_length() if wl.size else 1)
    index = pinned.empty(q.size, np.int32)
    dist = pinned.empty(q.size, np.uint8)
    devs = _devs(devices, q.size, MULTI_MIN_RECORDS)
    if devs:
        check(lib().sct_nearest_host_devices(kind, _ptr(wl), wl.size, _ptr(q), q.size, code_bits, max_d,
                                             _dev_array(devs), len(devs), _ptr(index), _ptr(dist)))
    else:
        check(lib().sct_nearest_host(kind, _ptr(wl), wl.size, _ptr(q), q.size, code_bits, max_d,
                                     _ptr(index), _ptr(dist)))
    return index, dist


class HostNearestPlan:
    """A nearest-whitelist plan built once from a host whitelist, queried with host arrays
    (sct_nearest_plan_create_host / sct_nearest_query_host): results in page-locked pool arrays.
    With several devices (``devices``, default set_devices()'s) the index is built on each and
    every query batch splits over them (sct_nearest_multi_*)."""

    def __init__(self, kind, whitelist, code_bits, max_d, devices=None):
        self._lib = lib()
        self._h = _vp()
        wl = np.ascontiguousarray(whitelist, dtype=np.uint64).reshape(-1)
        self.kind, self.nw, self.max_d = kind, wl.size, max_d
        devs = _devs(devices, 0, 0)
        self.devices = devs or [None]
        self._multi = bool(devs)
        if self._multi:
            check(self._lib.sct_nearest_multi_create_host(kind, _ptr(wl), wl.size, code_bits, max_d, _dev_array(devs),
                                                          len(devs), ctypes.byref(self._h)))
        else:
            check(self._lib.sct_nearest_plan_create_host(kind, _ptr(wl), wl.size, code_bits, max_d,
                                                         ctypes.byref(self._h)))

    def query(self, queries):
        q = np.ascontiguousarray(queries, dtype=np.uint64).reshape(-1)
        index = pinned.empty(q.size, np.int32)
        dist = pinned.empty(q.size, np.uint8)
        if q.size:
            f = self._lib.sct_nearest_multi_query_host if self._multi else self._lib.sct_nearest_query_host
            check(f(self._h, _ptr(q), q.size, _ptr(index), _ptr(dist)))
        return index, dist

    def close(self):
        if self._h:
            (self._lib.sct_nearest_multi_destroy if self._multi else self._lib.sct_nearest_plan_destroy)(self._h)
            self._h = _vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class NearestPlan:
    """Device-resident pigeonhole index of a whitelist (sct_nearest_plan)."""

    def __init__(self, kind, d_whitelist_ptr, nw, code_bits, max_d, stream=0):
        self._lib = lib()
        self._h = _vp()
        check(self._lib.sct_nearest_plan_create(kind, _vp(d_whitelist_ptr), nw, code_bits, max_d,
                                                _vp(stream), ctypes.byref(self._h)))

    def info(self):
        """dict(scheme: 'oa' | 'csr' | 'halves', index_bytes)."""
        sc, nb = _i32(0), _i64(0)
        check(self._lib.sct_nearest_plan_info(self._h, ctypes.byref(sc), ctypes.byref(nb)))
        return {"scheme": {1: "oa", 2: "csr", 3: "halves"}.get(sc.value, str(sc.value)), "index_bytes": nb.value}

    def query(self, d_queries_ptr, nq, d_index_ptr, d_dist_ptr, stream=0):
        check(self._lib.sct_nearest_query(self._h, _vp(d_queries_ptr), nq, _vp(d_index_ptr),
                                          _vp(d_dist_ptr), _vp(stream)))

    def close(self):
        if self._h:
            self._lib.sct_nearest_plan_destroy(self._h)
            self._h = _vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def device_count():
    c = _i32(0)
    rc = lib().sct_device_count(ctypes.byref(c))
    return c.value if rc == SCT_OK else 0


# ------------------------------------------------------------------ device-pointer plan API
class AllPairsPlan:
    """Owns an sct_allpairs_plan over device-resident codes (a torch.uint64/int64 tensor
    or a raw device pointer).  Used by the benchmark and the sharded driver.

    ``ncounts`` is the length of the uint64 counts vector that ``moments`` and ``count``
    accumulate into; ``counts_to_hist`` inverts the counts of the whole job."""

    def __init__(self, d_codes_ptr, n, code_bits=0, scheme=SCHEME_AUTO, distinct=False):
        self._lib = lib()
        self._h = _vp()
        check(self._lib.sct_allpairs_plan_create_ex2(_vp(d_codes_ptr), n, code_bits, scheme,
                                                     ALLPAIRS_DISTINCT if distinct else 0, ctypes.byref(self._h)))
        nb, items, pairs = _i32(0), _i64(0), _i64(0)
        check(self._lib.sct_allpairs_plan_info(self._h, ctypes.byref(nb), ctypes.byref(items), ctypes.byref(pairs)))
        self.nbins, self.items, self.pairs = nb.value, items.value, pairs.value
        sc, nc, cb = _i32(0), _i32(0), _i32(0)
        check(self._lib.sct_allpairs_plan_scheme(self._h, ctypes.byref(sc), ctypes.byref(nc), ctypes.byref(cb)))
        self.scheme, self.ncounts, self.code_bits = sc.value, nc.value, cb.value

    def build(self, stream=0, begin=None, end=None):
        """Selection table for items [begin, end) (default: all of them)."""
        if begin is None and end is None:
            check(self._lib.sct_allpairs_build(self._h, _vp(stream)))
        else:
            begin = 0 if begin is None else begin
            end = self.items if end is None else end
            check(self._lib.sct_allpairs_build_items(self._h, begin, end, _vp(stream)))

    def moments(self, d_counts_ptr, part=0, nparts=1, stream=0):
        """MOMENTS scheme: add moment share `part` of `nparts` (no-op for SUBSETS)."""
        check(self._lib.sct_allpairs_moments(self._h, part, nparts, _vp(d_counts_ptr), _vp(stream)))

    def count(self, d_counts_ptr, begin=0, end=None, grid=0, stream=0):
        end = self.items if end is None else end
        check(self._lib.sct_allpairs_count(self._h, begin, end, _vp(d_counts_ptr), grid, _vp(stream)))

    def counts_to_hist(self, counts):
        return counts_to_hist(counts, self.scheme, self.nbins)

    def time_kernels(self, d_scratch_ptr, begin=0, end=None, repeats=5, stream=0):
        """Bench aid: dict(kernel_ms, seed_ms, units) -- the dominant kernel's ms per launch
        (SPECTRAL: tile kernel on one chunk of `units` slices; else the count kernel)."""
        end = self.items if end is None else end
        out = (ctypes.c_double * 3)()
        check(self._lib.sct_allpairs_time_kernels(self._h, begin, end, _vp(d_scratch_ptr), repeats, out,
                                                  _vp(stream)))
        return {"kernel_ms": out[0], "seed_ms": out[1], "units": int(out[2])}

    def timing(self, mode):
        """Per-launch HIP-event timing of this plan's kernels (sct_allpairs_timing): mode 1
        start, 0 stop, 2 read.  Returns {kind: (ms summed, launches)} for seed, tile, count,
        build."""
        out = (ctypes.c_double * 8)()
        check(self._lib.sct_allpairs_timing(self._h, mode, out))
        return {k: (out[2 * i], int(out[2 * i + 1])) for i, k in enumerate(("seed", "tile", "count", "build"))}

    def spectral_info(self):
        """SPECTRAL plans: dict(elem_bytes, chunk_slices, max_column, column_bits)."""
        eb, ch, mc = _i32(0), _i64(0), _i32(0)
        check(self._lib.sct_allpairs_spectral_info(self._h, ctypes.byref(eb), ctypes.byref(ch), ctypes.byref(mc)))
        cb = _i32(0)
        check(self._lib.sct_allpairs_spectral_columns(self._h, ctypes.byref(cb)))
        return {"elem_bytes": eb.value, "chunk_slices": ch.value, "max_column": mc.value, "column_bits": cb.value}

    def range_pairs(self, begin, end):
        p = _i64(0)
        check(self._lib.sct_allpairs_range_pairs(self._h, begin, end, ctypes.byref(p)))
        return p.value

    def close(self):
        if self._h:
            self._lib.sct_allpairs_plan_destroy(self._h)
            self._h = _vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
