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
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <unistd.h>

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

/* Large plain dicts (CPython 3.10's combined table with no deleted entries, the layout below
 * checked against PyDict_Next before use) are read by kThreads threads, each a contiguous run
 * of the entries array: the loop is bound by streaming the entries and the int objects from
 * memory, one core at a time does ~12 GB/s of it (fewer threads when fewer CPUs are online).  The calling thread keeps the GIL for the
 * whole call and the workers only read (no reference counts, no Python API), so nothing can
 * change the dict under them.  Ints of up to three 30-bit digits are converted in place; any
 * other key ends a worker's run with the status the sequential loop would give it. */
#if PY_VERSION_HEX >= 0x030A0000 && PY_VERSION_HEX < 0x030B0000
#define SCT_PARALLEL_KEYS 1
#include <longintrepr.h> /* (3.10 only: from 3.11 it lives under cpython/ and Python.h has it) */
typedef struct {
  Py_hash_t me_hash;
  PyObject* me_key;
  PyObject* me_value;
} Entry310;
typedef struct {
  Py_ssize_t dk_refcnt;
  Py_ssize_t dk_size;
  void* dk_lookup;
  Py_ssize_t dk_usable;
  Py_ssize_t dk_nentries;
  char dk_indices[];
} Keys310;

/* 8 runs measured best on MI355X's host (737K keys: 0.38-0.43 ms against 0.39-0.57 with 4 and
 * 0.44-0.47 with 12; 3.3 ms for the sequential loop; profiles/ab_key_threads_r05.jsonl) */
enum { kThreads = 8, kParallelMin = 1 << 17 };

typedef struct {
  const Entry310* e;
  int64_t* out;
  Py_ssize_t b, end;  /* entries [b, end) into out[b, end) */
  Py_ssize_t stop;    /* first entry not converted (end when all were) */
  int status;
  int64_t lo, hi;
} Run;

static int conv_key(PyObject* k, int64_t* v) {
  if (!PyLong_Check(k)) return 1;
  const PyLongObject* L = (const PyLongObject*)k;
  const Py_ssize_t sz = Py_SIZE(k), a = sz < 0 ? -sz : sz;
  uint64_t u;
  if (a == 0)
    u = 0;
  else if (a == 1)
    u = L->ob_digit[0];
  else if (a == 2)
    u = (uint64_t)L->ob_digit[0] | ((uint64_t)L->ob_digit[1] << 30);
  else if (a == 3 && L->ob_digit[2] < 8)  /* < 2^63 */
    u = (uint64_t)L->ob_digit[0] | ((uint64_t)L->ob_digit[1] << 30) | ((uint64_t)L->ob_digit[2] << 60);
  else
    return 2;  /* (-2^63 too: the caller's general path takes it) */
  *v = sz < 0 ? -(int64_t)u : (int64_t)u;
  return 0;
}

static void* run_keys(void* arg) {
  Run* r = (Run*)arg;
  int64_t lo = INT64_MAX, hi = INT64_MIN;
  Py_ssize_t j = r->b;
  for (; j < r->end; ++j) {
    int64_t v;
    const int st = conv_key(r->e[j].me_key, &v);
    if (st) {
      r->status = st;
      break;
    }
    r->out[j] = v;
    if (v < lo) lo = v;
    if (v > hi) hi = v;
  }
  r->stop = j;
  r->lo = lo;
  r->hi = hi;
  return NULL;
}

/* 1 and (status, count, lo, hi) when the parallel form ran, 0 when it does not apply */
static int keys_parallel(PyObject* d, int64_t* out, Py_ssize_t cap, int* status, Py_ssize_t* count, int64_t* lo,
                         int64_t* hi) {
  PyDictObject* mp = (PyDictObject*)d;
  const Py_ssize_t n = mp->ma_used;
  if (n < kParallelMin || n > cap || mp->ma_values != NULL) return 0;
  const Keys310* dk = (const Keys310*)mp->ma_keys;
  if (dk->dk_nentries != n) return 0;  /* deleted entries: holes in the array */
  const Py_ssize_t size = dk->dk_size;
  const int ix = size <= 0xff ? 1 : size <= 0xffff ? 2 : size <= 0xffffffffLL ? 4 : 8;
  const Entry310* e = (const Entry310*)(&dk->dk_indices[size * ix]);
  /* the layout is what this code assumes: the first and the last key as PyDict_Next sees them */
  Py_ssize_t pos = 0;
  PyObject *k, *v;
  if (!PyDict_Next(d, &pos, &k, &v) || k != e[0].me_key || v != e[0].me_value) return 0;
  if (e[n - 1].me_key == NULL || e[n - 1].me_value == NULL) return 0;
  pos = n - 1;
  if (!PyDict_Next(d, &pos, &k, &v) || k != e[n - 1].me_key || PyDict_Next(d, &pos, &k, &v)) return 0;
  /* the CPUs this process may run on (affinity mask / cpuset), not the machine's: a pinned or
   * quota-limited caller gets no more threads than it has CPUs, and one CPU the plain loop */
  long cpus = 1;
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof(set), &set) == 0)
    cpus = CPU_COUNT(&set);
  else
    cpus = sysconf(_SC_NPROCESSORS_ONLN);
  if (cpus <= 1) return 0;
  const int T = cpus >= kThreads ? kThreads : (int)cpus;
  Run runs[kThreads];
  pthread_t tid[kThreads];
  int started[kThreads] = {0};
  for (int t = 0; t < T; ++t) {
    runs[t] = (Run){e, out, n * t / T, n * (t + 1) / T, 0, 0, 0, 0};
    if (t > 0) started[t] = pthread_create(&tid[t], NULL, run_keys, &runs[t]) == 0;
  }
  run_keys(&runs[0]);
  for (int t = 1; t < T; ++t) {
    if (started[t])
      pthread_join(tid[t], NULL);
    else
      run_keys(&runs[t]);  /* (no thread: this one does the run) */
  }
  *status = 0;
  *count = n;
  *lo = INT64_MAX;
  *hi = INT64_MIN;
  for (int t = 0; t < T; ++t) {  /* the first run that stopped decides, as the sequential loop */
    if (runs[t].lo < *lo) *lo = runs[t].lo;
    if (runs[t].hi > *hi) *hi = runs[t].hi;
    if (runs[t].status) {
      *status = runs[t].status;
      *count = runs[t].stop;
      break;
    }
  }
  return 1;
}
#endif

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
#ifdef SCT_PARALLEL_KEYS
  if (PyDict_Check(keys) && keys_parallel(keys, out, cap, &status, &i, &lo, &hi)) {
    /* (lo / hi cover the keys before the first stop, as below) */
  } else
#endif
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
