/*
 * ORACLE — test infrastructure only.  C restatement of the reference's pair loop
 * (src/sctools/barcode.py:42-43 calling TwoBit.hamming_distance,
 * src/sctools/encodings.py:113-121).  Used by tests/ (parity at sizes the Python
 * reference cannot reach), __graft_entry__.smoke() and bench.py's cpu_baseline leg;
 * never linked into libsctools_hip.so.  Pinned against tests/golden/ by
 * tests/test_oracle_golden.py.
 */
#include <stdint.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* encodings.py:113-121, statement for statement: XOR, then walk 2-bit groups. */
static inline int hamming_scalar(uint64_t a, uint64_t b) {
  uint64_t diff = a ^ b;
  int d = 0;
  while (diff) {
    if (diff & 3u) d += 1;
    diff >>= 2;
  }
  return d;
}

/* The same count in closed form: non-zero 2-bit groups of x = popcount((x|x>>1) & 0x55..). */
static inline int hamming_popcnt(uint64_t a, uint64_t b) {
  const uint64_t x = a ^ b;
  return __builtin_popcountll((x | (x >> 1)) & 0x5555555555555555ull);
}

int oracle_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

/* hist[d] += #pairs (i, j) with row_begin <= i < row_end, i < j < n (1 core, scalar loop). */
void oracle_hist_scalar(const uint64_t* codes, int64_t n, int64_t row_begin, int64_t row_end,
                        int64_t* hist) {
  for (int64_t i = row_begin; i < row_end && i < n; ++i)
    for (int64_t j = i + 1; j < n; ++j) hist[hamming_scalar(codes[i], codes[j])] += 1;
}

/* Same pairs, popcount form, OpenMP over rows (threads <= 0: OpenMP default). */
void oracle_hist_popcnt(const uint64_t* codes, int64_t n, int64_t row_begin, int64_t row_end,
                        int64_t* hist, int threads) {
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#endif
  if (row_end > n) row_end = n;
#pragma omp parallel
  {
    int64_t local[65];
    memset(local, 0, sizeof(local));
#pragma omp for schedule(dynamic, 16)
    for (int64_t i = row_begin; i < row_end; ++i) {
      const uint64_t a = codes[i];
      for (int64_t j = i + 1; j < n; ++j) local[hamming_popcnt(a, codes[j])] += 1;
    }
#pragma omp critical
    for (int d = 0; d < 65; ++d) hist[d] += local[d];
  }
}

/* Pairs of work items [t0, t1) in the kernel's chunk-major enumeration: item (c, r) =
 * rows [r*rb, (r+1)*rb) x columns [c*cb, (c+1)*cb), pairs i < j < n.  Independent of
 * the device code: enumerates chunks and their row counts directly. */
void oracle_hist_items(const uint64_t* codes, int64_t n, int64_t rb, int64_t cb, int64_t* hist,
                       int64_t t0, int64_t t1, int64_t* pairs, int threads) {
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#endif
  int64_t t = 0, np_ = 0;
  const int64_t nchunks = (n + cb - 1) / cb;
  for (int64_t c = 0; c < nchunks && t < t1; ++c) {
    int64_t maxj = ((c + 1) * cb < n ? (c + 1) * cb : n) - 1;
    int64_t rows = maxj <= 0 ? 0 : (maxj + rb - 1) / rb;
    for (int64_t r = 0; r < rows; ++r, ++t) {
      if (t < t0 || t >= t1) continue;
      const int64_t ilo = r * rb, ihi = (r + 1) * rb < n ? (r + 1) * rb : n;
      const int64_t jlo = c * cb, jhi = (c + 1) * cb < n ? (c + 1) * cb : n;
#pragma omp parallel for reduction(+ : np_) schedule(static)
      for (int64_t i = ilo; i < ihi; ++i) {
        int64_t local[65];
        memset(local, 0, sizeof(local));
        for (int64_t j = (jlo > i + 1 ? jlo : i + 1); j < jhi; ++j) {
          local[hamming_popcnt(codes[i], codes[j])] += 1;
          np_ += 1;
        }
#pragma omp critical
        for (int d = 0; d < 65; ++d) hist[d] += local[d];
      }
    }
  }
  *pairs = np_;
}
