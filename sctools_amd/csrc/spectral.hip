// Spectral all-pairs scheme: the TwoBit distance histogram of n 16-base codes from the
// Walsh-Hadamard transform of their multiplicity f over Z_2^32.
//
//   d(x, y) = digit weight of x ^ y (non-zero 2-bit digits), so the ordered-pair counts
//   N(d) = sum_{v : wt(v) = d} R(v), R = f (*) f (XOR autocorrelation), and with
//   F = WHT(f):  N(d) = 2^-32 sum_z F(z)^2 K_d(wt(z)),  K_d the q = 4 Krawtchouk
//   polynomial.  The device computes S_w = sum_{wt(z) = w} F(z)^2 (17 uint64); the host
//   (sct_counts_to_hist_ex) applies K and halves: hist[d] = (N(d) - n [d = 0]) / 2.
//
// Work does not depend on n: 2^32 int32 transform values, 64 GB of HBM traffic per
// job, cut into 4096 slices of 2^20 values (z >> 20), the plan's work items.  Per slice:
//   seed      z's high 12 bits, straight from the codes (F's inner sums are short:
//             ~n / 2^20 codes share each low-20-bit value) -> write 4 MB
//   tile      butterflies over bits 0..13 in LDS (64 KB contiguous tiles) -> r+w 8 MB
//   square    butterflies over bits 14..19 in registers, F^2 binned by digit weight
//             -> read 4 MB, no write
// Exact: |F| <= n < 2^31 in int32, F^2 and S_w in uint64 (S_w <= 2^32 sum f^2).
#include <hipcub/hipcub.hpp>

#include "sct_common.h"
#include "spectral.h"

namespace sct_spectral {
namespace {

constexpr int kLo = 1 << kLoBits;
constexpr int kTileBits = 14;  // tile pass: lo bits 0..13
constexpr int kTile = 1 << kTileBits;
constexpr int kTilesPerSlice = kLo / kTile;  // 64 = the square pass's register transform
constexpr int kSeedZ = 64;     // slices per seed workgroup (16 per wave)
constexpr int kRegCodes = 8;   // per-lane codes held in registers by the seed

// non-zero 2-bit digits of z
__device__ __forceinline__ int digit_weight(uint32_t z) {
  return __popc((z | (z >> 1)) & 0x55555555u);
}
constexpr int digit_weight_c(uint32_t z) {
  int w = 0;
  for (; z; z >>= 2) w += (z & 3) != 0;
  return w;
}

// in-register WHT of N values
template <int N>
__device__ __forceinline__ void wht(int32_t* x) {
#pragma unroll
  for (int h = 1; h < N; h <<= 1)
#pragma unroll
    for (int i = 0; i < N; ++i)
      if (!(i & h)) {
        const int32_t a = x[i], b = x[i | h];
        x[i] = a + b;
        x[i | h] = a - b;
      }
}

// off[k] = first index whose low 20 bits are >= k (k = 0..2^20), hi[i] = sorted[i] >> 20
__global__ void split_kernel(const uint64_t* __restrict__ sorted, int64_t n, uint16_t* __restrict__ hi,
                             uint32_t* __restrict__ off) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t < n) hi[t] = (uint16_t)(sorted[t] >> kLoBits);
  if (t <= kLo) {
    int64_t a = 0, b = n;
    while (a < b) {
      const int64_t m = (a + b) >> 1;
      if ((int64_t)(sorted[m] & (kLo - 1)) < t) a = m + 1;
      else b = m;
    }
    off[t] = (uint32_t)a;
  }
}

// buf[(z - z0) 2^20 + lo] = sum over codes c with c & (2^20-1) = lo of (-1)^popc((c >> 20) & z)
// A wave holds 64 consecutive lo (256 B rows) and loops over 16 slices.
__global__ __launch_bounds__(256) void seed_kernel(const uint16_t* __restrict__ hi,
                                                   const uint32_t* __restrict__ off, int z0, int z1,
                                                   int32_t* __restrict__ buf) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lo = blockIdx.x * 64 + lane;
  const uint32_t b = off[lo];
  const int cnt = (int)(off[lo + 1] - b);
  int wmax = cnt;
#pragma unroll
  for (int s = 32; s; s >>= 1) wmax = max(wmax, __shfl_xor(wmax, s));
  uint32_t h[kRegCodes];
#pragma unroll
  for (int j = 0; j < kRegCodes; ++j) h[j] = j < cnt ? hi[b + j] : 0u;  // 0: parity 0
  const int zb = z0 + (int)blockIdx.y * kSeedZ;
  const int ze = min(zb + kSeedZ, z1);
  for (int z = zb + wave; z < ze; z += 4) {
    int par = 0;
#pragma unroll
    for (int j = 0; j < kRegCodes; ++j)
      if (j < wmax) par += __popc(h[j] & (uint32_t)z) & 1;
    for (int j = kRegCodes; j < wmax; ++j)  // crowded low-bit values only
      if (j < cnt) par += __popc((uint32_t)hi[b + j] & (uint32_t)z) & 1;
    buf[(int64_t)(z - z0) * kLo + lo] = cnt - 2 * par;
  }
}

// LDS word of tile element i: 4-word groups of a 64-word row XOR-swizzled by the row,
// so row-parallel (phase 2) b128 reads take the minimum 4 passes and every
// column-parallel access is conflict-free.
__device__ __forceinline__ int swz(int i) { return i ^ (((i >> 6) & 15) << 2); }

// WHT over bits 0..13 of each 2^14-value tile, in place.
__global__ __launch_bounds__(256) void tile_kernel(int32_t* __restrict__ buf) {
  __shared__ int32_t lds[kTile];
  int32_t* t = buf + (int64_t)blockIdx.x * kTile;
  const int tid = threadIdx.x;
  int32_t x[64];
  // phase 1: bits 8..13 (thread = bits 0..7)
#pragma unroll
  for (int k = 0; k < 64; ++k) x[k] = __builtin_nontemporal_load(t + k * 256 + tid);
  wht<64>(x);
#pragma unroll
  for (int k = 0; k < 64; ++k) lds[swz(k * 256 + tid)] = x[k];
  __syncthreads();
  // phase 2: bits 0..5 (thread = bits 6..13)
#pragma unroll
  for (int j = 0; j < 64; j += 4) {
    const int4 v = *reinterpret_cast<const int4*>(lds + swz(tid * 64 + j));
    x[j] = v.x;
    x[j + 1] = v.y;
    x[j + 2] = v.z;
    x[j + 3] = v.w;
  }
  wht<64>(x);
#pragma unroll
  for (int j = 0; j < 64; j += 4)
    *reinterpret_cast<int4*>(lds + swz(tid * 64 + j)) = make_int4(x[j], x[j + 1], x[j + 2], x[j + 3]);
  __syncthreads();
  // phase 3: bits 6, 7 (thread = bits 0..5 and 8, 9; loop over bits 10..13)
  const int l = tid & 63, w = tid >> 6;
#pragma unroll
  for (int c = 0; c < 16; ++c)
#pragma unroll
    for (int a = 0; a < 4; ++a) x[c * 4 + a] = lds[swz(c * 1024 + w * 256 + a * 64 + l)];
#pragma unroll
  for (int c = 0; c < 16; ++c) wht<4>(x + c * 4);
#pragma unroll
  for (int c = 0; c < 16; ++c)
#pragma unroll
    for (int a = 0; a < 4; ++a) t[c * 1024 + w * 256 + a * 64 + l] = x[c * 4 + a];
}

// WHT over bits 14..19, then S_w += F^2 by digit weight w; slices [z0, z0 + nslices).
// Persistent: workgroups stride over (slice, 256-column) units; 17 global atomics each.
__global__ __launch_bounds__(256) void square_kernel(const int32_t* __restrict__ buf, int z0,
                                                     int nslices,
                                                     unsigned long long* __restrict__ counts) {
  __shared__ unsigned long long bins[17];
  const int tid = threadIdx.x;
  if (tid < 17) bins[tid] = 0;
  __syncthreads();
  const int64_t units = (int64_t)nslices * (kTile / 256);
  for (int64_t u = blockIdx.x; u < units; u += gridDim.x) {
    const int s = (int)(u / (kTile / 256));
    const int col = (int)(u % (kTile / 256)) * 256 + tid;  // lo bits 0..13
    const int32_t* p = buf + (int64_t)s * kLo + col;
    int32_t x[kTilesPerSlice];
#pragma unroll
    for (int m = 0; m < kTilesPerSlice; ++m) x[m] = __builtin_nontemporal_load(p + m * kTile);
    wht<kTilesPerSlice>(x);
    unsigned long long acc[4] = {0, 0, 0, 0};
#pragma unroll
    for (int m = 0; m < kTilesPerSlice; ++m)
      acc[digit_weight_c(m)] += (unsigned long long)((int64_t)x[m] * x[m]);
    const int w0 = digit_weight(((uint32_t)(z0 + s) << kLoBits) | (uint32_t)col);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (acc[k]) atomicAdd(&bins[w0 + k], acc[k]);
  }
  __syncthreads();
  if (tid < 17 && bins[tid]) atomicAdd(counts + 1 + tid, bins[tid]);
}

__global__ void add_kernel(unsigned long long* p, unsigned long long v) { atomicAdd(p, v); }

}  // namespace

int create(State& st, int64_t n, int64_t chunk, int cus) {
  st.n = n;
  st.chunk = std::max<int64_t>(1, std::min<int64_t>(chunk, kSlices));
  st.grid = std::max(1, cus) * 8;
  if (n < 2) return SCT_OK;
  SCT_HIP(hipMalloc(&st.d_sorted, (size_t)n * 8));
  SCT_HIP(hipMalloc(&st.d_hi, (size_t)n * 2));
  SCT_HIP(hipMalloc(&st.d_off, (size_t)(kLo + 1) * 4));
  SCT_HIP(hipMalloc(&st.d_buf, (size_t)st.chunk * kLo * 4));
  SCT_HIP(hipcub::DeviceRadixSort::SortKeys(nullptr, st.sort_tmp_bytes, (const uint64_t*)nullptr,
                                            (uint64_t*)nullptr, (int)n, 0, kLoBits));
  SCT_HIP(hipMalloc(&st.d_sort_tmp, std::max<size_t>(st.sort_tmp_bytes, 16)));
  return SCT_OK;
}

void destroy(State& st) {
  for (void* p : {(void*)st.d_sorted, (void*)st.d_hi, (void*)st.d_off, (void*)st.d_buf, st.d_sort_tmp})
    if (p) (void)hipFree(p);
  st = State();
}

int build(State& st, const uint64_t* d_codes, hipStream_t s) {
  if (st.n < 2) return SCT_OK;
  size_t bytes = st.sort_tmp_bytes;
  SCT_HIP(hipcub::DeviceRadixSort::SortKeys(st.d_sort_tmp, bytes, d_codes, st.d_sorted, (int)st.n, 0,
                                            kLoBits, s));
  const int64_t threads = std::max<int64_t>(st.n, kLo + 1);
  hipLaunchKernelGGL(split_kernel, dim3((unsigned)sct::ceil_div(threads, 256)), dim3(256), 0, s,
                     st.d_sorted, st.n, st.d_hi, st.d_off);
  SCT_LAUNCH_CHECK();
  return SCT_OK;
}

int count(State& st, int64_t z_begin, int64_t z_end, unsigned long long* d_counts, hipStream_t s) {
  SCT_CHECK(0 <= z_begin && z_begin <= z_end && z_end <= kSlices, "slice range [%lld, %lld)",
            (long long)z_begin, (long long)z_end);
  if (st.n < 2 || z_begin == z_end) return SCT_OK;
  for (int64_t z0 = z_begin; z0 < z_end; z0 += st.chunk) {
    const int z1 = (int)std::min<int64_t>(z_end, z0 + st.chunk);
    const int ns = z1 - (int)z0;
    hipLaunchKernelGGL(seed_kernel, dim3(kLo / 64, (unsigned)sct::ceil_div(ns, kSeedZ)), dim3(256), 0, s,
                       st.d_hi, st.d_off, (int)z0, z1, st.d_buf);
    SCT_LAUNCH_CHECK();
    hipLaunchKernelGGL(tile_kernel, dim3((unsigned)(ns * kTilesPerSlice)), dim3(256), 0, s, st.d_buf);
    SCT_LAUNCH_CHECK();
    const int grid = (int)std::min<int64_t>(st.grid, (int64_t)ns * (kTile / 256));
    hipLaunchKernelGGL(square_kernel, dim3(grid), dim3(256), 0, s, st.d_buf, (int)z0, ns, d_counts);
    SCT_LAUNCH_CHECK();
  }
  if (z_begin == 0) {
    hipLaunchKernelGGL(add_kernel, dim3(1), dim3(1), 0, s, d_counts, (unsigned long long)st.n);
    SCT_LAUNCH_CHECK();
  }
  return SCT_OK;
}

}  // namespace sct_spectral
