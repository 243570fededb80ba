/*
 * ORACLE — test infrastructure only.  C restatement of the reference's pair loop
 * (src/sctools/barcode.py:42-43 calling TwoBit.hamming_distance,
 * src/sctools/encodings.py:113-121).  Used by tests/ (parity at sizes the Python
 * reference cannot reach), __graft_entry__.smoke() and bench.py's cpu_baseline leg;
 * never linked into libsctools_hip.so.  Pinned against tests/golden/ by
 * tests/test_oracle_golden.py.
 */
#include <stdint.h>
#include <stdlib.h>
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

/* ---- 16-base fast path: the same popcount form over 32-bit lanes, 16 pairs per AVX-512
 * vector (bench.py's cpu_baseline and the full-size parity tests; distances d <= 16).
 * Counting without a scatter: every lane adds 1 << 4d into a nibble accumulator (bins
 * 0..7) and 1 << 4(d-8) into a second one (bins 8..15; a shift of 32 or more gives 0, so
 * d = 16 falls out of both and is recovered from the pair count).  Nibbles are spilled to
 * byte fields every 15 vectors and bytes to int64 every 17 spills (15 * 17 = 255). */
#if defined(__x86_64__)
#include <immintrin.h>
#include <stdlib.h>

__attribute__((target("avx512f,avx512bw,avx512vpopcntdq"))) static void hist16_row_avx512(
    const uint32_t* c, int64_t n, int64_t i, int64_t* hist) {
  const __m512i a = _mm512_set1_epi32((int)c[i]);
  const __m512i m55 = _mm512_set1_epi32(0x55555555);
  const __m512i one = _mm512_set1_epi32(1);
  const __m512i m0f = _mm512_set1_epi32(0x0F0F0F0F);
  const __m512i mff = _mm512_set1_epi32(0xFF);
  const __m512i k32 = _mm512_set1_epi32(32);
  __m512i b8[4]; /* byte accumulators: bins 0..7 even / odd, bins 8..15 even / odd */
  for (int k = 0; k < 4; ++k) b8[k] = _mm512_setzero_si512();
  int64_t j = i + 1, vpairs = 0, binned = 0;
  for (; j < n && (j & 15); ++j) hist[hamming_popcnt(c[i], c[j])] += 1;
  int spills = 0;
  while (j + 16 <= n) {
    __m512i lo = _mm512_setzero_si512(), hi = _mm512_setzero_si512();
    int v = 0;
    for (; v < 15 && j + 16 <= n; ++v, j += 16) {
      const __m512i x = _mm512_xor_si512(a, _mm512_load_si512((const void*)(c + j)));
      const __m512i y = _mm512_and_si512(_mm512_or_si512(x, _mm512_srli_epi32(x, 1)), m55);
      const __m512i d4 = _mm512_slli_epi32(_mm512_popcnt_epi32(y), 2);
      lo = _mm512_add_epi32(lo, _mm512_sllv_epi32(one, d4));
      hi = _mm512_add_epi32(hi, _mm512_sllv_epi32(one, _mm512_sub_epi32(d4, k32)));
    }
    vpairs += 16 * v;
    b8[0] = _mm512_add_epi32(b8[0], _mm512_and_si512(lo, m0f));
    b8[1] = _mm512_add_epi32(b8[1], _mm512_and_si512(_mm512_srli_epi32(lo, 4), m0f));
    b8[2] = _mm512_add_epi32(b8[2], _mm512_and_si512(hi, m0f));
    b8[3] = _mm512_add_epi32(b8[3], _mm512_and_si512(_mm512_srli_epi32(hi, 4), m0f));
    if (++spills == 17 || j + 16 > n) {
      /* byte f of accumulator k holds bin 8 (k >> 1) + 2 f + (k & 1) */
      for (int k = 0; k < 4; ++k) {
        for (int f = 0; f < 4; ++f) {
          const int64_t s = _mm512_reduce_add_epi32(_mm512_and_si512(_mm512_srli_epi32(b8[k], 8 * f), mff));
          hist[8 * (k >> 1) + 2 * f + (k & 1)] += s;
          binned += s;
        }
        b8[k] = _mm512_setzero_si512();
      }
      spills = 0;
    }
  }
  hist[16] += vpairs - binned; /* d = 16 added nothing to either accumulator */
  for (; j < n; ++j) hist[hamming_popcnt(c[i], c[j])] += 1;
}

static int have_vpopcnt(void) {
  __builtin_cpu_init();
  return __builtin_cpu_supports("avx512vpopcntdq") && __builtin_cpu_supports("avx512bw");
}
#endif

/* hist[d] += #pairs (i, j), row_begin <= i < row_end, i < j < n, for codes < 2^32 (the
 * 16-base TwoBit case).  Returns 1 if the AVX-512 path ran, 0 if it fell back to
 * oracle_hist_popcnt (no VPOPCNTDQ, or a code >= 2^32). */
int oracle_hist16(const uint64_t* codes, int64_t n, int64_t row_begin, int64_t row_end, int64_t* hist,
                  int threads) {
#if defined(__x86_64__)
  int ok = have_vpopcnt();
  for (int64_t i = 0; ok && i < n; ++i) ok = codes[i] < (1ull << 32);
  if (!ok) {
    oracle_hist_popcnt(codes, n, row_begin, row_end, hist, threads);
    return 0;
  }
  uint32_t* c = (uint32_t*)aligned_alloc(64, (size_t)((n + 16) * 4 + 63) / 64 * 64);
  if (!c) {
    oracle_hist_popcnt(codes, n, row_begin, row_end, hist, threads);
    return 0;
  }
  for (int64_t i = 0; i < n; ++i) c[i] = (uint32_t)codes[i];
  if (row_end > n) row_end = n;
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#endif
#pragma omp parallel
  {
    int64_t local[65];
    memset(local, 0, sizeof(local));
#pragma omp for schedule(dynamic, 64)
    for (int64_t i = row_begin; i < row_end; ++i) {
      hist16_row_avx512(c, n, i, local);
    }
#pragma omp critical
    for (int d = 0; d < 65; ++d) hist[d] += local[d];
  }
  free(c);
  return 1;
#else
  oracle_hist_popcnt(codes, n, row_begin, row_end, hist, threads);
  return 0;
#endif
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

/* Multi-limb codes (Python ints >= 2^64 as `words` little-endian uint64 limbs): the same
 * TwoBit distance of encodings.py:113-121 -- 2-bit groups never straddle a 64-bit limb, so
 * it is the sum of the per-limb counts.  hist must hold 32 * words + 1 bins. */
void oracle_hist_wide(const uint64_t* codes, int64_t n, int words, int64_t* hist, int threads) {
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#endif
  const int nb = 32 * words + 1;
#pragma omp parallel
  {
    int64_t* local = (int64_t*)calloc((size_t)nb, sizeof(int64_t));
#pragma omp for schedule(dynamic, 16)
    for (int64_t i = 0; i < n; ++i) {
      const uint64_t* a = codes + i * words;
      for (int64_t j = i + 1; j < n; ++j) {
        const uint64_t* b = codes + j * words;
        int d = 0;
        for (int w = 0; w < words; ++w) d += hamming_popcnt(a[w], b[w]);
        local[d] += 1;
      }
    }
#pragma omp critical
    for (int d = 0; d < nb; ++d) hist[d] += local[d];
    free(local);
  }
}

/* Brute-force nearest whitelist entry (the contract of sct_nearest_*; no reference
 * function exists) under the reference's distance: kind 2 =
 * TwoBit.hamming_distance (encodings.py:113-121), kind 3 = ThreeBit.hamming_distance
 * (encodings.py:194-202).  index[i] = the unique j at the minimal distance <= max_d, -2 for
 * a tie, -1 for none; dist[i] = that distance or 255.  OpenMP over queries. */
static inline int hamming3_popcnt(uint64_t a, uint64_t b) {
  const uint64_t x = a ^ b;
  return __builtin_popcountll((x | (x >> 1) | (x >> 2)) & 0x9249249249249249ull);
}

void oracle_nearest(int kind, const uint64_t* wl, int64_t nw, const uint64_t* q, int64_t nq, int max_d,
                    int32_t* index, uint8_t* dist, int threads) {
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#endif
#pragma omp parallel for schedule(dynamic, 64)
  for (int64_t i = 0; i < nq; ++i) {
    const uint64_t a = q[i];
    int best = 1 << 30;
    int64_t arg = -1, ties = 0;
    for (int64_t j = 0; j < nw; ++j) {
      const int d = kind == 2 ? hamming_popcnt(a, wl[j]) : hamming3_popcnt(a, wl[j]);
      if (d < best) {
        best = d;
        arg = j;
        ties = 1;
      } else if (d == best) {
        ties += 1;
      }
    }
    if (arg >= 0 && best <= max_d) {
      index[i] = ties == 1 ? (int32_t)arg : -2;
      dist[i] = (uint8_t)best;
    } else {
      index[i] = -1;
      dist[i] = 255;
    }
  }
}
