// Host-side logic of libsctools_hip.so: error state, device selection, the exact
// subset-count -> histogram inversion and the bit-exact numpy summary.
#include <math.h>
#include <string.h>

#include <sched.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <utility>
#include <vector>

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

HostStage* host_stage() {
  static thread_local HostStage* stages[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
    fail(SCT_E_HIP, "host stage: no current device");
    return nullptr;
  }
  if (!stages[dev]) {
    auto* st = new HostStage();
    st->device = dev;
    if (hipStreamCreateWithFlags(&st->stream, hipStreamNonBlocking) != hipSuccess) {
      fail(SCT_E_HIP, "host stage: hipStreamCreate failed");
      delete st;
      return nullptr;
    }
    stages[dev] = st;
  }
  return stages[dev];
}

void stage_release_device() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return;
  HostStage* st = host_stage();
  if (!st || !st->dev) return;
  (void)hipStreamSynchronize(st->stream);
  (void)hipFree(st->dev);
  st->dev = nullptr;
  st->dev_cap = 0;
}

// ---------------------------------------------------------------- parallel host copies
// The pageable side of the host streams: one core copies ~10 GB/s, a PCIe 5 x16 link moves ~57, so
// a chunk's copy into (or out of) the page-locked stage is split over helper threads.  The helpers
// are created once (never destroyed: they wait until the process exits); a copy that finds them
// busy (another thread's stream) runs on the calling thread alone.
namespace {
struct CopyPool {
  std::mutex call_mu, mu;
  std::condition_variable go, done;
  uint64_t gen = 0;
  int nthreads = 0, pending = 0;
  uint8_t* dst = nullptr;
  const uint8_t* src = nullptr;
  size_t bytes = 0;
  int parts = 1;
  static void part(uint8_t* d, const uint8_t* s, size_t bytes, int r, int parts) {
    const size_t a = (bytes * r / parts) & ~(size_t)63, b = r + 1 == parts ? bytes : (bytes * (r + 1) / parts) & ~(size_t)63;
    if (b > a) memcpy(d + a, s + a, b - a);
  }
  void loop(int r) {
    uint64_t seen = 0;
    for (;;) {
      std::unique_lock<std::mutex> lk(mu);
      go.wait(lk, [&] { return gen != seen; });
      seen = gen;
      if (r + 1 >= parts) continue;  // (slot 0 is the caller)
      uint8_t* d = dst;
      const uint8_t* sr = src;
      const size_t b = bytes;
      const int k = parts;
      lk.unlock();
      part(d, sr, b, r + 1, k);
      lk.lock();
      if (--pending == 0) done.notify_all();
    }
  }
};
CopyPool* copy_pool() {
  static CopyPool* p = new CopyPool();
  return p;
}
int copy_helpers() {
  static const int h = [] {
    cpu_set_t set;
    int cpus = sched_getaffinity(0, sizeof(set), &set) == 0 ? CPU_COUNT(&set) : 1;
    return std::max(0, std::min(7, cpus / 2 - 1));  // (leave the other half to the caller's own work)
  }();
  return h;
}
}  // namespace

void par_memcpy(void* dst, const void* src, size_t bytes) {
  const int helpers = copy_helpers();
  CopyPool* p = copy_pool();
  if (bytes < ((size_t)4 << 20) || helpers == 0 || !p->call_mu.try_lock()) {
    memcpy(dst, src, bytes);
    return;
  }
  std::lock_guard<std::mutex> call(p->call_mu, std::adopt_lock);
  const int parts = (int)std::min<size_t>((size_t)helpers + 1, bytes >> 21);  // >= 2 MiB per part
  {
    std::lock_guard<std::mutex> lk(p->mu);
    while (p->nthreads < helpers) {
      const int r = p->nthreads++;
      std::thread([p, r] { p->loop(r); }).detach();
    }
    p->dst = static_cast<uint8_t*>(dst);
    p->src = static_cast<const uint8_t*>(src);
    p->bytes = bytes;
    p->parts = parts;
    p->pending = parts - 1;
    ++p->gen;
  }
  p->go.notify_all();
  CopyPool::part(static_cast<uint8_t*>(dst), static_cast<const uint8_t*>(src), bytes, 0, parts);
  std::unique_lock<std::mutex> lk(p->mu);
  p->done.wait(lk, [&] { return p->pending == 0; });
}

bool host_range_pinned(const void* p, size_t bytes) {
  if (!p || !bytes) return false;
  hipPointerAttribute_t a{};
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  if (a.type != hipMemoryTypeHost) return false;
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  if (hipMemGetAddressRange(&base, &size, const_cast<void*>(p)) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  const uintptr_t b = reinterpret_cast<uintptr_t>(base), q = reinterpret_cast<uintptr_t>(p);
  return q >= b && q - b <= size && bytes <= size - (q - b);
}

int stage_reserve(HostStage* st, size_t pinned_bytes, size_t dev_bytes) {
  auto grow = [](size_t have, size_t need) {
    size_t c = have ? have : (size_t)1 << 16;
    while (c < need) c *= 2;
    return c;
  };
  if (pinned_bytes > st->pinned_cap) {
    if (st->pinned) (void)hipHostFree(st->pinned);
    st->pinned = nullptr;
    st->pinned_cap = 0;
    const size_t c = grow(0, pinned_bytes);
    SCT_HIP(hipHostMalloc((void**)&st->pinned, c, hipHostMallocCoherent | hipHostMallocMapped));
    SCT_HIP(hipHostGetDevicePointer((void**)&st->pinned_dev, st->pinned, 0));
    st->pinned_cap = c;
  }
  if (dev_bytes > st->dev_cap) {
    if (st->dev) (void)hipFree(st->dev);
    st->dev = nullptr;
    st->dev_cap = 0;
    const size_t c = grow(0, dev_bytes);
    SCT_HIP(hipMalloc((void**)&st->dev, c));
    st->dev_cap = c;
  }
  return SCT_OK;
}

// Launch-shape knobs (sct_tune_set), stored as value + 1 (0 = unset: zero-initialised
// before any constructor runs).  The library reads no environment variable; nothing here
// changes a result.
static std::atomic<int64_t> g_tune[SCT_TUNE_NKEYS];

int64_t tune(int key, int64_t dflt) {
  if (key <= 0 || key >= SCT_TUNE_NKEYS) return dflt;
  const int64_t v = g_tune[key].load(std::memory_order_relaxed);
  return v == 0 ? dflt : v - 1;
}

// The library's own stream-ordered memory pool per device (the device's DEFAULT
// pool, which PyTorch and other libraries share, is left alone).  Its release threshold is
// raised once, so per-call scratch is reused from the pool instead of being mapped and unmapped
// around every stream synchronisation.
static std::mutex g_pool_mu;
static hipMemPool_t g_pools[64] = {};

static hipMemPool_t existing_pool(int dev) {
  std::lock_guard<std::mutex> lk(g_pool_mu);
  return dev >= 0 && dev < 64 ? g_pools[dev] : nullptr;
}

static hipMemPool_t private_pool(int dev) {
  static bool tried[64] = {};
  hipMemPool_t* pools = g_pools;
  if (dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> lk(g_pool_mu);
  if (!tried[dev]) {
    tried[dev] = true;
    hipMemPoolProps props = {};
    props.allocType = hipMemAllocationTypePinned;
    props.handleTypes = hipMemHandleTypeNone;
    props.location.type = hipMemLocationTypeDevice;
    props.location.id = dev;
    hipMemPool_t pool = nullptr;
    if (hipMemPoolCreate(&pool, &props) == hipSuccess) {
      uint64_t keep = UINT64_MAX;
      (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
      pools[dev] = pool;
    } else {
      (void)hipGetLastError();
    }
  }
  return pools[dev];
}

hipError_t pool_alloc(void** p, size_t bytes, hipStream_t s) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  bytes = bytes ? bytes : 1;
  hipMemPool_t pool = private_pool(dev);
  return pool ? hipMallocFromPoolAsync(p, bytes, pool, s) : hipMallocAsync(p, bytes, s);
}

void pool_free(void* p, hipStream_t s) {
  if (p) (void)hipFreeAsync(p, s);
}

// hands the idle memory of every pool created so far back to the device (the callers have
// synchronised the work that freed it)
void pool_trim() {
  for (int dev = 0; dev < 64; ++dev)
    if (hipMemPool_t pool = existing_pool(dev)) (void)hipMemPoolTrimTo(pool, 0);
}

}  // namespace sct

extern "C" int sct_tune_set(int key, int64_t value) {
  SCT_CHECK(key > 0 && key < SCT_TUNE_NKEYS, "unknown tuning key %d", key);
  sct::g_tune[key].store(value < 0 ? 0 : value + 1);
  return SCT_OK;
}

extern "C" int sct_tune_get(int key, int64_t* value) {
  SCT_CHECK(key > 0 && key < SCT_TUNE_NKEYS, "unknown tuning key %d", key);
  SCT_CHECK(value != nullptr, "value is NULL");
  *value = sct::tune(key, -1);
  return SCT_OK;
}

extern "C" int sct_host_pinned(const void* p, int64_t bytes, int* pinned) {
  SCT_CHECK(pinned != nullptr && bytes >= 0, "bad arguments");
  *pinned = sct::host_range_pinned(p, (size_t)bytes) ? 1 : 0;
  return SCT_OK;
}

extern "C" int sct_host_alloc(int64_t bytes, void** ptr) {
  SCT_CHECK(ptr != nullptr && bytes > 0, "bad arguments");
  *ptr = nullptr;
  const hipError_t e = hipHostMalloc(ptr, (size_t)bytes, hipHostMallocDefault);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    *ptr = nullptr;
    return sct::fail(SCT_E_NOMEM, "hipHostMalloc(%lld): %s", (long long)bytes, hipGetErrorString(e));
  }
  return SCT_OK;
}

extern "C" int sct_host_free(void* ptr) {
  if (ptr) SCT_HIP(hipHostFree(ptr));
  return SCT_OK;
}

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

// ---------------------------------------------------------------- MOMENTS inversion
// The 17 MOMENTS functionals of hist[0..16] (counts layout in sctools_hip.h):
//   row 0: 1 (pairs);  rows 1..13: prod of bits kMomProducts[r-1] of (d mod 16);
//   rows 14..16: C(16 - d, k), k = 1..3 (agreement moments).
// A is fixed and non-singular, so hist = adj(A) counts / det(A).  adj and det come from a
// fraction-free (Bareiss) Gauss-Jordan elimination of [A | I] in __int128 (every division
// is exact; |minors| < 1e14), checked once against A adj(A) = det I.
namespace {

constexpr int kN = sct::kMomNCounts;
static_assert(kN == sct::kMomG + 1, "MOMENTS system must be square");

int64_t binom(int64_t a, int k) {
  if (a < k) return 0;
  int64_t r = 1;
  for (int j = 0; j < k; ++j) r = r * (a - j) / (j + 1);
  return r;
}

int64_t mom_row(int r, int d) {
  if (r == 0) return 1;
  if (r <= sct::kMomNProd) {
    const int m = sct::kMomProducts[r - 1];
    return ((d & 15) & m) == m ? 1 : 0;
  }
  return binom(sct::kMomG - d, r - sct::kMomNProd);
}

struct MomInverse {
  bool ok = false;
  __int128 det = 0;
  __int128 adj[kN][kN];  // A^-1 = adj / det (row i of adj gives hist[i])
  MomInverse() {
    __int128 M[kN][2 * kN];
    for (int i = 0; i < kN; ++i)
      for (int j = 0; j < 2 * kN; ++j)
        M[i][j] = j < kN ? (__int128)mom_row(i, j) : (__int128)(j - kN == i);
    __int128 prev = 1;
    for (int k = 0; k < kN; ++k) {
      int p = k;
      while (p < kN && M[p][k] == 0) ++p;
      if (p == kN) return;  // singular
      if (p != k)
        for (int j = 0; j < 2 * kN; ++j) std::swap(M[p][j], M[k][j]);
      for (int i = 0; i < kN; ++i) {
        if (i == k) continue;
        for (int j = 0; j < 2 * kN; ++j) {
          if (j == k) continue;
          const __int128 v = M[k][k] * M[i][j] - M[i][k] * M[k][j];
          if (v % prev != 0) return;  // not exact: refuse rather than round
          M[i][j] = v / prev;
        }
        M[i][k] = 0;
      }
      prev = M[k][k];
    }
    // every diagonal entry now equals det (up to the row swaps' sign, already applied)
    det = M[kN - 1][kN - 1];
    for (int i = 0; i < kN; ++i) {
      if (M[i][i] != det) return;
      for (int j = 0; j < kN; ++j) adj[i][j] = M[i][kN + j];
    }
    // check A adj = det I
    for (int i = 0; i < kN; ++i)
      for (int j = 0; j < kN; ++j) {
        __int128 s = 0;
        for (int t = 0; t < kN; ++t) s += (__int128)mom_row(i, t) * adj[t][j];
        if (s != (i == j ? det : 0)) return;
      }
    ok = det != 0;
  }
};

const MomInverse& mom_inverse() {
  static const MomInverse inv;  // thread-safe one-time init
  return inv;
}

}  // namespace

// SPECTRAL counts [n, sum f^2, S_w limbs 0 / 1 / 2] (spectral.h) -> hist.  Ordered pairs
// (self pairs included) at distance d: N(d) = 2^-32 sum_w S_w K_d(w), K_d(w) = [t^d]
// (1 + 3t)^(16-w) (1 - t)^w (per 2-bit digit: 3 non-zero XOR values, characters sum to 3 if
// z's digit is 0, else -1); hist[d] = (N(d) - n [d = 0]) / 2.  Every step is checked exact,
// and against the independently computed sum f^2: S_0 = F(0)^2 = n^2 and, by Parseval,
// sum_w S_w = 2^32 sum f^2 -- a wrap of any S_w (mod 2^64) would break the latter.
static int spectral_to_hist(const uint64_t* counts, int ncounts, uint64_t* hist, int nbins) {
  constexpr int G = 16;
  constexpr int kLimb0 = 2, kLimb1 = kLimb0 + G + 1, kLimb2 = kLimb1 + G + 1, kCounts = kLimb2 + G + 1;
  SCT_CHECK(ncounts == kCounts && nbins == G + 1, "SPECTRAL counts/hist hold %d/%d values (got %d, %d)",
            kCounts, G + 1, ncounts, nbins);
  __int128 S[G + 1];
  unsigned __int128 sum_s = 0;
  for (int w = 0; w <= G; ++w) {
    // every limb is a sum of < 2^32 pieces (or small high words): none can be near 2^63
    const uint64_t l0 = counts[kLimb0 + w], l1 = counts[kLimb1 + w], l2 = counts[kLimb2 + w];
    SCT_CHECK(l0 < (1ull << 62) && l1 < (1ull << 62) && l2 < (1ull << 40),
              "inconsistent SPECTRAL counts (limbs of S_%d)", w);
    const unsigned __int128 v = (unsigned __int128)l0 + ((unsigned __int128)l1 << 32) + ((unsigned __int128)l2 << 64);
    S[w] = (__int128)v;
    sum_s += v;
  }
  const __int128 n = counts[0];
  const unsigned __int128 sumsq = counts[1];
  if (S[0] != n * n)
    return sct::fail(SCT_E_RANGE, "inconsistent SPECTRAL counts (S_0 != n^2)");
  if (n >= 2 && (sumsq < (unsigned __int128)n || sum_s != (sumsq << 32)))
    return sct::fail(SCT_E_RANGE, "inconsistent SPECTRAL counts (sum_w S_w != 2^32 sum f^2)");
  struct Kraw {
    __int128 k[G + 1][G + 1];  // k[d][w]
    Kraw() {
      for (int w = 0; w <= G; ++w) {
        __int128 poly[G + 1] = {1};
        for (int f = 0; f < G; ++f) {  // multiply by (1 + 3t) or (1 - t)
          const int c = f < G - w ? 3 : -1;
          for (int d = G; d >= 1; --d) poly[d] += c * poly[d - 1];
        }
        for (int d = 0; d <= G; ++d) k[d][w] = poly[d];
      }
    }
  };
  static const Kraw kraw;
  const auto& K = kraw.k;
  __int128 total = 0;
  for (int d = 0; d <= G; ++d) {
    __int128 s = 0;  // |K| < 3^16, S_w <= 2^32 n^2 <= 2^86 (n <= 1e8): no overflow
    for (int w = 0; w <= G; ++w) s += K[d][w] * S[w];
    if (s % ((__int128)1 << 32) != 0)
      return sct::fail(SCT_E_RANGE, "inconsistent SPECTRAL counts (bin %d not integral)", d);
    __int128 h = s >> 32;
    if (d == 0) h -= n;
    if (h < 0 || (h & 1))
      return sct::fail(SCT_E_RANGE, "inconsistent SPECTRAL counts (bin %d)", d);
    h >>= 1;
    if (h > (__int128)UINT64_MAX) return sct::fail(SCT_E_RANGE, "SPECTRAL bin %d out of range", d);
    hist[d] = (uint64_t)h;
    total += h;
  }
  if (total != n * (n - 1) / 2)
    return sct::fail(SCT_E_RANGE, "inconsistent SPECTRAL counts (pair total)");
  return SCT_OK;
}

extern "C" int sct_counts_to_hist_ex(int scheme, const uint64_t* counts, int ncounts,
                                     uint64_t* hist, int nbins) {
  SCT_CHECK(counts && hist, "NULL pointer");
  if (scheme == SCT_ALLPAIRS_SUBSETS) {
    SCT_CHECK(ncounts == nbins, "SUBSETS counts hold nbins values (%d != %d)", ncounts, nbins);
    return sct_counts_to_hist(counts, nbins, hist);
  }
  if (scheme == SCT_ALLPAIRS_SPECTRAL) return spectral_to_hist(counts, ncounts, hist, nbins);
  SCT_CHECK(scheme == SCT_ALLPAIRS_MOMENTS, "unknown scheme %d", scheme);
  SCT_CHECK(ncounts == kN && nbins == kN, "MOMENTS counts/hist hold %d values (got %d, %d)", kN,
            ncounts, nbins);
  const MomInverse& inv = mom_inverse();
  if (!inv.ok) return sct::fail(SCT_E_HIP, "MOMENTS system inverse unavailable");
  for (int i = 0; i < kN; ++i) {
    __int128 s = 0;
    for (int j = 0; j < kN; ++j) s += inv.adj[i][j] * (__int128)counts[j];
    if (s % inv.det != 0)
      return sct::fail(SCT_E_RANGE, "inconsistent MOMENTS counts (bin %d not integral)", i);
    const __int128 h = s / inv.det;
    if (h < 0 || h > (__int128)UINT64_MAX)
      return sct::fail(SCT_E_RANGE, "inconsistent MOMENTS counts (bin %d out of range)", i);
    hist[i] = (uint64_t)h;
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
