// Host-side logic of libsctools_hip.so: error state, device selection, the exact
// subset-count -> histogram inversion and the bit-exact numpy summary.
#include <math.h>
#include <string.h>

#include "sct_common.h"

namespace sct {

static thread_local char g_err[1024] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

const char* last_error() { return g_err; }

}  // namespace sct

extern "C" int sct_version(void) { return 1; }

extern "C" const char* sct_last_error(void) { return sct::last_error(); }

extern "C" int sct_device_count(int* count) {
  SCT_CHECK(count != nullptr, "count is NULL");
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess) {
    *count = 0;
    return sct::fail(SCT_E_HIP, "hipGetDeviceCount: %s", hipGetErrorString(e));
  }
  *count = c;
  return SCT_OK;
}

extern "C" int sct_set_device(int device) {
  SCT_HIP(hipSetDevice(device));
  return SCT_OK;
}

// counts[m] = #pairs whose distance d satisfies (d & m) == m, counts[0] = #pairs.
// Every d < nbins, so counts of masks >= nbins are 0 and the subset-lattice Moebius
// inversion over 2^B masks recovers hist exactly:
//   hist[d] = sum_{m superset of d} (-1)^{|m \ d|} counts[m].
extern "C" int sct_counts_to_hist(const uint64_t* counts, int nbins, uint64_t* hist) {
  SCT_CHECK(counts && hist, "NULL pointer");
  SCT_CHECK(nbins >= 1 && nbins <= 129, "nbins %d out of range", nbins);
  int B = 0;
  while ((1 << B) < nbins) ++B;
  const int M = 1 << B;
  int64_t f[256];
  for (int m = 0; m < M; ++m) f[m] = m < nbins ? (int64_t)counts[m] : 0;
  for (int b = 0; b < B; ++b)
    for (int m = 0; m < M; ++m)
      if (!(m & (1 << b))) f[m] -= f[m | (1 << b)];
  for (int m = nbins; m < M; ++m)
    if (f[m] != 0) return sct::fail(SCT_E_RANGE, "inconsistent subset counts (mask %d)", m);
  for (int d = 0; d < nbins; ++d) {
    if (f[d] < 0) return sct::fail(SCT_E_RANGE, "inconsistent subset counts (bin %d < 0)", d);
    hist[d] = (uint64_t)f[d];
  }
  return SCT_OK;
}

// Order statistic os(k) (0-based) of the multiset described by hist.
static int64_t order_stat(const uint64_t* hist, int nbins, uint64_t k) {
  uint64_t cum = 0;
  for (int d = 0; d < nbins; ++d) {
    cum += hist[d];
    if (k < cum) return d;
  }
  return nbins - 1;  // unreachable for k < total
}

// numpy 2.x np.percentile(a, q*100), method='linear', on an int64 array:
//   v = (n-1)*q; if v >= n-1: a[-1]; else lerp(a[floor v], a[floor v + 1], v - floor v)
// with numpy's _lerp: a + (b-a)*t, replaced by b - (b-a)*(1-t) where t >= 0.5
// (numpy/lib/_function_base_impl.py: _QuantileMethods['linear'], _get_indexes, _lerp).
static double percentile_linear(const uint64_t* hist, int nbins, uint64_t n, double q) {
  const double v = (double)(n - 1) * q;
  if (v >= (double)(n - 1)) return (double)order_stat(hist, nbins, n - 1);
  const double prev = floor(v);
  const uint64_t p = (uint64_t)prev;
  const double g = v - prev;
  const int64_t a = order_stat(hist, nbins, p);
  const int64_t b = order_stat(hist, nbins, p + 1);
  const double diff = (double)(b - a);
  double r = (double)a + diff * g;
  if (g >= 0.5) r = (double)b - diff * (1.0 - g);
  return r;
}

extern "C" int sct_summary_from_hist(const uint64_t* hist, int nbins, double* out) {
  SCT_CHECK(hist && out, "NULL pointer");
  SCT_CHECK(nbins >= 1, "nbins must be >= 1");
  uint64_t n = 0;
  unsigned __int128 s = 0;
  for (int d = 0; d < nbins; ++d) {
    n += hist[d];
    s += (unsigned __int128)hist[d] * (unsigned)d;
  }
  if (n == 0) return sct::fail(SCT_E_RANGE, "index -1 is out of bounds for axis 0 with size 0");
  if (n >= (1ull << 53) || s >= ((unsigned __int128)1 << 53))
    return sct::fail(SCT_E_RANGE, "histogram too large for an exact float64 mean");
  static const double qs[5] = {0.0, 0.25, 0.5, 0.75, 1.0};
  for (int i = 0; i < 5; ++i) out[i] = percentile_linear(hist, nbins, n, qs[i]);
  // np.mean on ints: float64 pairwise sum (exact, every partial sum < 2^53) / float64(n)
  out[5] = (double)(uint64_t)s / (double)n;
  return SCT_OK;
}
