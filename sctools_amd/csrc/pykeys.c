/* CPython helper of Barcodes.codes_array (sctools_amd/barcode.py): the keys of the barcode
 * mapping into an int64 buffer in one C loop.  The reference's pair loop (barcode.py:42-43 ->
 * encodings.py:113-121) takes `a ^ b` of the keys, so only integers are valid keys; the
 * Python-side conversion (a per-key type scan, then np.fromiter) was 12 ms of the 16.8-ms
 * drop-in call at 737K keys (profiles/single_call_breakdown_r03.json).  This loop does the type
 * check and the conversion together and leaves every other case to the Python path:
 *
 *   keys_to_int64(mapping_or_iterable, out) -> (status, count, min, max)
 *     status 0: every key is a Python int (bool and int subclasses included) within int64,
 *               out[0:count] holds them in iteration order
 *     status 1: a key is not a Python int (numpy scalars, floats, str, ...): the caller's
 *               general path decides (TypeError as the reference, or numpy integers)
 *     status 2: an int outside int64 (the caller's multi-limb path)
 *     status 3: more keys than out holds (the mapping changed size)
 *   min / max: of out[0:count] (0, 0 when count is 0), taken in the same pass so the caller
 *   needs no numpy reduction over the keys for the sign check and the code width
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>

static int put_key(PyObject* k, int64_t* out, Py_ssize_t cap, Py_ssize_t* i, int64_t* lo, int64_t* hi) {
  if (!PyLong_Check(k)) return 1;
  int ovf = 0;
  const long long v = PyLong_AsLongLongAndOverflow(k, &ovf);
  if (ovf) return 2;
  if (v == -1 && PyErr_Occurred()) {
    PyErr_Clear();
    return 2;
  }
  if (*i >= cap) return 3;
  out[(*i)++] = (int64_t)v;
  if (v < *lo) *lo = v;
  if (v > *hi) *hi = v;
  return 0;
}

static PyObject* keys_to_int64(PyObject* self, PyObject* args) {
  (void)self;
  PyObject* keys;
  Py_buffer buf;
  if (!PyArg_ParseTuple(args, "Ow*", &keys, &buf)) return NULL;
  int64_t* out = (int64_t*)buf.buf;
  const Py_ssize_t cap = buf.len / (Py_ssize_t)sizeof(int64_t);
  Py_ssize_t i = 0;
  int status = 0;
  int64_t lo = INT64_MAX, hi = INT64_MIN;
  if (PyDict_Check(keys)) {  /* dict / Counter: the storage in insertion (= keys()) order */
    Py_ssize_t pos = 0;
    PyObject *k, *v;
    while (status == 0 && PyDict_Next(keys, &pos, &k, &v)) status = put_key(k, out, cap, &i, &lo, &hi);
  } else {
    PyObject* it = PyObject_GetIter(keys);
    if (!it) {
      PyBuffer_Release(&buf);
      return NULL;
    }
    PyObject* k;
    while (status == 0 && (k = PyIter_Next(it)) != NULL) {
      status = put_key(k, out, cap, &i, &lo, &hi);
      Py_DECREF(k);
    }
    Py_DECREF(it);
    if (PyErr_Occurred()) {
      PyBuffer_Release(&buf);
      return NULL;
    }
  }
  PyBuffer_Release(&buf);
  if (i == 0) lo = hi = 0;
  return Py_BuildValue("(inLL)", status, i, (long long)lo, (long long)hi);
}

static PyMethodDef kMethods[] = {
    {"keys_to_int64", keys_to_int64, METH_VARARGS, "keys -> int64 buffer; returns (status, count, min, max)"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_pykeys", NULL, -1, kMethods, NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__pykeys(void) { return PyModule_Create(&kModule); }
