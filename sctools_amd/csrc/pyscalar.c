/* CPython entry points of the drop-in's scalar methods (TwoBit / ThreeBit .encode, .decode,
 * .gc_content, .hamming_distance: encodings.py:75-121, 155-202), each a batch of one through the
 * library's *_host calls and its resident scalar server (encode.hip).
 *
 * The ctypes path cost about 1.1 us per call on top of the 2.1-us C call (argument conversion,
 * thread-local buffers, addressof, the status check: profiles/scalar_floor_r06/), about as much
 * as the reference's whole pure-Python hamming_distance.  These functions take the common case
 * -- Python ints in [0, 2^64), a bytes record of one limb -- straight to the C call with the
 * buffers on the C stack, and return NotImplemented for everything else (other types, negative
 * or multi-limb codes, an ambiguous base, a library error), which the Python method then hands
 * to its general path: that path keeps the reference's semantics and raises the errors.
 *
 * The library's entry points are bound once it is loaded (_lib.lib() calls bind() with their
 * addresses); until then every function returns NotImplemented.  The GIL is released around the
 * C call, as ctypes does (the scalar server is per host thread).
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>
#include <string.h>

typedef int (*hamming_fn)(int, const uint64_t*, const uint64_t*, int64_t, int, int32_t*);
typedef int (*gc_fn)(int, const uint64_t*, int64_t, int, int, int32_t*);
typedef int (*decode2_fn)(const uint64_t*, int64_t, int, int, uint8_t*);
typedef int (*encode_fn)(int, const uint8_t*, int64_t, int64_t, int, uint64_t*, uint8_t*, uint8_t*);
typedef int (*decode3_fn)(const uint64_t*, int64_t, int, int, uint8_t*, int32_t*, int32_t*);

static hamming_fn g_hamming;
static gc_fn g_gc;
static decode2_fn g_decode2;
static encode_fn g_encode;
static decode3_fn g_decode3;

static PyObject* not_impl(void) { Py_RETURN_NOTIMPLEMENTED; }

/* 1 and *v when o is a Python int (bool and int subclasses included) in [0, 2^64), else 0 */
static int as_u64(PyObject* o, uint64_t* v) {
  if (!PyLong_Check(o)) return 0;
  const unsigned long long x = PyLong_AsUnsignedLongLong(o);
  if (x == (unsigned long long)-1 && PyErr_Occurred()) { /* negative or >= 2^64 */
    PyErr_Clear();
    return 0;
  }
  *v = (uint64_t)x;
  return 1;
}

static int as_int(PyObject* o, int* v) {
  if (!PyLong_Check(o)) return 0;
  const long x = PyLong_AsLong(o);
  if (x == -1 && PyErr_Occurred()) {
    PyErr_Clear();
    return 0;
  }
  if (x < -2147483647L || x > 2147483647L) return 0;
  *v = (int)x;
  return 1;
}

static PyObject* bind(PyObject* self, PyObject* args) {
  unsigned long long h, g, d, e, d3;
  if (!PyArg_ParseTuple(args, "KKKKK", &h, &g, &d, &e, &d3)) return NULL;
  g_hamming = (hamming_fn)(uintptr_t)h;
  g_gc = (gc_fn)(uintptr_t)g;
  g_decode2 = (decode2_fn)(uintptr_t)d;
  g_encode = (encode_fn)(uintptr_t)e;
  g_decode3 = (decode3_fn)(uintptr_t)d3;
  Py_RETURN_NONE;
}

/* hamming(kind, a, b) -> int: hamming_distance of two one-limb codes (encodings.py:113-121 / 194-202) */
static PyObject* hamming(PyObject* self, PyObject* const* args, Py_ssize_t n) {
  int kind;
  uint64_t a, b;
  if (n != 3 || !g_hamming || !as_int(args[0], &kind) || !as_u64(args[1], &a) || !as_u64(args[2], &b))
    return not_impl();
  int32_t out = 0;
  int rc;
  Py_BEGIN_ALLOW_THREADS
  rc = g_hamming(kind, &a, &b, 1, 1, &out);
  Py_END_ALLOW_THREADS
  if (rc != 0) return not_impl();
  return PyLong_FromLong(out);
}

/* gc(kind, code, L) -> int: gc_content of a one-limb code (encodings.py:102-111 / 182-192) */
static PyObject* gc(PyObject* self, PyObject* const* args, Py_ssize_t n) {
  int kind, L;
  uint64_t x;
  if (n != 3 || !g_gc || !as_int(args[0], &kind) || !as_u64(args[1], &x) || !as_int(args[2], &L) || L < 0 ||
      (kind == 2 && L == 0))
    return not_impl();
  int32_t out = 0;
  int rc;
  Py_BEGIN_ALLOW_THREADS
  rc = g_gc(kind, &x, 1, 1, L, &out);
  Py_END_ALLOW_THREADS
  if (rc != 0) return not_impl();
  return PyLong_FromLong(out);
}

/* decode2(code, L) -> bytes: TwoBit(L).decode of a one-limb code, 1 <= L <= 64 (encodings.py:90-100) */
static PyObject* decode2(PyObject* self, PyObject* const* args, Py_ssize_t n) {
  int L;
  uint64_t x;
  if (n != 2 || !g_decode2 || !as_u64(args[0], &x) || !as_int(args[1], &L) || L < 1 || L > 64) return not_impl();
  uint8_t out[64];
  int rc;
  Py_BEGIN_ALLOW_THREADS
  rc = g_decode2(&x, 1, 1, L, out);
  Py_END_ALLOW_THREADS
  if (rc != 0) return not_impl();
  return PyBytes_FromStringAndSize((const char*)out, L);
}

/* decode3(code) -> bytes: ThreeBit.decode of a one-limb code (encodings.py:169-180); NotImplemented
 * when a triplet has no base (the Python path raises the reference's KeyError) */
static PyObject* decode3(PyObject* self, PyObject* const* args, Py_ssize_t n) {
  uint64_t x;
  if (n != 1 || !g_decode3 || !as_u64(args[0], &x)) return not_impl();
  enum { kMax = 22 }; /* ceil(64 / 3) triplets */
  uint8_t out[kMax];
  int32_t len = 0, bad = -1;
  int rc;
  Py_BEGIN_ALLOW_THREADS
  rc = g_decode3(&x, 1, 1, kMax, out, &len, &bad);
  Py_END_ALLOW_THREADS
  if (rc != 0 || bad >= 0 || len < 0 || len > kMax) return not_impl();
  return PyBytes_FromStringAndSize((const char*)out + (kMax - len), len);
}

/* encode(kind, seq) -> int: TwoBit / ThreeBit .encode of a bytes record of one limb (1..32 / 1..21
 * bytes; encodings.py:75-88 / 155-167); NotImplemented when a TwoBit record has an ambiguous or
 * invalid base (the Python path draws the random bases in order or raises the KeyError) */
static PyObject* encode(PyObject* self, PyObject* const* args, Py_ssize_t n) {
  int kind;
  if (n != 2 || !g_encode || !as_int(args[0], &kind) || (kind != 2 && kind != 3) || !PyBytes_CheckExact(args[1]))
    return not_impl();
  const Py_ssize_t L = PyBytes_GET_SIZE(args[1]);
  if (L < 1 || L > (kind == 2 ? 32 : 21)) return not_impl();
  uint8_t seq[32];
  memcpy(seq, PyBytes_AS_STRING(args[1]), (size_t)L);
  uint64_t code = 0;
  uint8_t flags = 0;
  int rc;
  Py_BEGIN_ALLOW_THREADS
  rc = g_encode(kind, seq, 1, (int64_t)L, (int)L, &code, NULL, &flags);
  Py_END_ALLOW_THREADS
  if (rc != 0 || (kind == 2 && flags)) return not_impl();
  return PyLong_FromUnsignedLongLong(code);
}

static PyMethodDef methods[] = {
    {"bind", bind, METH_VARARGS, "bind(hamming, gc, decode2, encode, decode3): the library entry points' addresses"},
    {"hamming", (PyCFunction)(void (*)(void))hamming, METH_FASTCALL, "hamming(kind, a, b) -> int or NotImplemented"},
    {"gc", (PyCFunction)(void (*)(void))gc, METH_FASTCALL, "gc(kind, code, L) -> int or NotImplemented"},
    {"decode2", (PyCFunction)(void (*)(void))decode2, METH_FASTCALL, "decode2(code, L) -> bytes or NotImplemented"},
    {"decode3", (PyCFunction)(void (*)(void))decode3, METH_FASTCALL, "decode3(code) -> bytes or NotImplemented"},
    {"encode", (PyCFunction)(void (*)(void))encode, METH_FASTCALL, "encode(kind, seq) -> int or NotImplemented"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_scalar", NULL, -1, methods};

PyMODINIT_FUNC PyInit__scalar(void) { return PyModule_Create(&module); }
