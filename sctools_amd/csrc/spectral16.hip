// SPECTRAL on 16-bit columns ("16-bit columns"): the same histogram as
// spectral.hip -- S_w = sum_{wt(z) = w} F(z)^2, F = WHT of the codes' multiplicity over Z_2^32 --
// for sets too dense for int8 seeds on 14-bit columns (config 5: 3.69M codes, ~225 per 14-bit
// column, int16 seeds).  Split z = (slice z >> 16, column z & 0xFFFF) instead: ~56 codes per
// column, so the seeds are int8 again (the plan requires <= 127 codes in every 16-bit column),
// a column has at most 4 groups of 32 codes, and the seed -> tile intermediate stays 1 byte per
// value: 1 GiB per 16,384 slices of 64 KiB.
//
//   seed   as seed_body in spectral.hip with 16 bit planes per group (four 16-B words)
//   tile   one WORKGROUP per 64-KiB slice, wave s holding column digit 7 (bits 14, 15) = s:
//          each wave runs the register tile of spectral.hip over its 16 KiB (two 64-point
//          MFMA stages over column digits 0-5 and Parseval over digit 6 = R), and digit 7
//          (across the waves) is handled by Parseval too.  With G_rs the 12-bit transform of
//          plane (R = r, S = s), T_s = sum_r G_rs, U_r = sum_s G_rs, V = sum G_rs, per (P', Q'):
//            [R' = 0, S' = 0]               V^2
//            one of R', S' non-zero         4 sum_r U_r^2 + 4 sum_s T_s^2 - 2 V^2
//            both non-zero                  16 sum G^2 - 4 sum U^2 - 4 sum T^2 + V^2
//          G and T_s are each wave's own (as in spectral.hip); U_r needs all four waves: every
//          wave adds its stage-1 outputs of plane r into an LDS image of U_r (ds_add_u32 on
//          biased int16 pairs, no carry), and after a barrier wave q takes quarter q (P' bits
//          4, 5) of every U_r through stage 2 (the two-byte split of spectral.hip); V's
//          transform is the sum of the four U_r transforms.
// Build: the 2^16 columns keep per-workgroup counts and scatter cursors as packed bytes in
// LDS (every column holds <= 127 codes, so no byte carries), 64 KB per workgroup.
#include <algorithm>
#include <vector>

#include "sct_common.h"
#include "spectral.h"

namespace sct_spectral {
namespace {

constexpr int kLo16 = 1 << kLoBits16;               // columns
constexpr int kHi16 = kSpaceBits - kLoBits16;       // 16 bit planes
constexpr int kPW16 = 16;                           // plane words per group: four 16-B words
constexpr int kWalk16 = 64, kWalkBits16 = 6;
constexpr int kSeedWalks16 = 16;
constexpr int kSortWGs16 = 128, kSortThreads16 = 1024;
constexpr int kChunk16 = kSlices16;                 // at most every real slice in one seed / tile pass: 4 GiB

__device__ __forceinline__ void wg_range16(int64_t n, int64_t& b, int64_t& e) {
  b = n * blockIdx.x / gridDim.x;
  e = n * (blockIdx.x + 1) / gridDim.x;
}

// ---------------------------------------------------------------- build
// workgroup g: byte counts of its contiguous share of the codes per column -> H[g][.] (bytes)
__global__ __launch_bounds__(kSortThreads16) void hist16_wg_kernel(const uint64_t* __restrict__ codes, int64_t n,
                                                                   uint32_t* __restrict__ H) {
  __shared__ uint32_t h[kLo16 / 4];
  for (int w = threadIdx.x; w < kLo16 / 4; w += kSortThreads16) h[w] = 0;
  __syncthreads();
  int64_t b, e;
  wg_range16(n, b, e);
  for (int64_t i = b + threadIdx.x; i < e; i += kSortThreads16) {
    const uint32_t c = (uint32_t)codes[i] & (kLo16 - 1);
    atomicAdd(&h[c >> 2], 1u << (8 * (c & 3)));
  }
  __syncthreads();
  uint32_t* out = H + (int64_t)blockIdx.x * (kLo16 / 4);
  for (int w = threadIdx.x; w < kLo16 / 4; w += kSortThreads16) out[w] = h[w];
}

// per 4 columns (one word of bytes): H[g] <- exclusive prefix over the workgroups, m(c) = totals
__global__ __launch_bounds__(256) void prefix16_kernel(uint32_t* __restrict__ H, int wgs, uint32_t* __restrict__ m) {
  const int w = blockIdx.x * 256 + threadIdx.x;
  uint32_t run = 0;
#pragma unroll 8
  for (int g = 0; g < wgs; ++g) {
    const uint32_t v = H[(int64_t)g * (kLo16 / 4) + w];
    H[(int64_t)g * (kLo16 / 4) + w] = run;
    run += v;  // bytes: every column total <= 127
  }
  reinterpret_cast<uint4*>(m)[w] = make_uint4(run & 255, (run >> 8) & 255, (run >> 16) & 255, run >> 24);
}

// one workgroup of 1024: 64 columns per thread; off / gofs = exclusive scans of m and ceil(m / 32)
__global__ __launch_bounds__(1024) void scan16_kernel(const uint32_t* __restrict__ m, uint32_t* __restrict__ off,
                                                      uint32_t* __restrict__ gofs) {
  constexpr int PT = kLo16 / 1024;
  __shared__ uint32_t wsum[2][16];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const uint32_t* mt = m + t * PT;
  uint32_t s = 0, sg = 0;
  for (int k = 0; k < PT; k += 4) {
    const uint4 q = *reinterpret_cast<const uint4*>(mt + k);
    s += q.x + q.y + q.z + q.w;
    sg += (q.x + 31) / 32 + (q.y + 31) / 32 + (q.z + 31) / 32 + (q.w + 31) / 32;
  }
  uint32_t is = s, isg = sg;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t a = __shfl_up(is, d), ag = __shfl_up(isg, d);
    if (lane >= d) {
      is += a;
      isg += ag;
    }
  }
  if (lane == 63) {
    wsum[0][wave] = is;
    wsum[1][wave] = isg;
  }
  __syncthreads();
  uint32_t run = is - s, rung = isg - sg;
  for (int w = 0; w < wave; ++w) {
    run += wsum[0][w];
    rung += wsum[1][w];
  }
  for (int k = 0; k < PT; k += 4) {
    const uint4 q = *reinterpret_cast<const uint4*>(mt + k);
    const uint32_t v[4] = {q.x, q.y, q.z, q.w};
    uint32_t o[4], og[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o[j] = run;
      og[j] = rung;
      run += v[j];
      rung += (v[j] + 31) / 32;
    }
    *reinterpret_cast<uint4*>(off + t * PT + k) = make_uint4(o[0], o[1], o[2], o[3]);
    *reinterpret_cast<uint4*>(gofs + t * PT + k) = make_uint4(og[0], og[1], og[2], og[3]);
  }
  if (t == 1023) {
    off[kLo16] = run;
    gofs[kLo16] = rung;
  }
}

// workgroup g: byte cursors (its prefix H[g]) in LDS, one LDS atomic per code
__global__ __launch_bounds__(kSortThreads16) void scatter16_wg_kernel(const uint64_t* __restrict__ codes, int64_t n,
                                                                      const uint32_t* __restrict__ H,
                                                                      const uint32_t* __restrict__ off,
                                                                      uint32_t* __restrict__ hi) {
  __shared__ uint32_t cur[kLo16 / 4];
  const uint32_t* pre = H + (int64_t)blockIdx.x * (kLo16 / 4);
  for (int w = threadIdx.x; w < kLo16 / 4; w += kSortThreads16) cur[w] = pre[w];
  __syncthreads();
  int64_t b, e;
  wg_range16(n, b, e);
  for (int64_t i = b + threadIdx.x; i < e; i += kSortThreads16) {
    const uint64_t x = codes[i];
    const uint32_t c = (uint32_t)x & (kLo16 - 1), sh = 8 * (c & 3);
    const uint32_t slot = (atomicAdd(&cur[c >> 2], 1u << sh) >> sh) & 255u;
    hi[off[c] + slot] = (uint32_t)(x >> kLoBits16);
  }
}

// planes of group slot k (< 4) of column c: 16 words, plane b bit j = bit b of (code >> 16)
// of the group's j-th code
__global__ __launch_bounds__(256) void planes16_kernel(const uint32_t* __restrict__ hi, const uint32_t* __restrict__ off,
                                                       const uint32_t* __restrict__ gofs, uint32_t* __restrict__ planes) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int c = t >> 2, k = t & 3;
  const uint32_t g0 = gofs[c];
  if (k >= (int)(gofs[c + 1] - g0)) return;
  const uint32_t first = off[c] + 32u * k, last = min(first + 32u, off[c + 1]);
  uint32_t p[kHi16];
#pragma unroll
  for (int b = 0; b < kHi16; ++b) p[b] = 0;
  for (uint32_t i = first; i < last; ++i) {
    const uint32_t h = hi[i], bit = 1u << (i - first);
#pragma unroll
    for (int b = 0; b < kHi16; ++b) p[b] |= (h >> b) & 1u ? bit : 0u;
  }
  uint4* q = reinterpret_cast<uint4*>(planes + (int64_t)(g0 + k) * kPW16);
#pragma unroll
  for (int i = 0; i < 4; ++i) q[i] = make_uint4(p[4 * i], p[4 * i + 1], p[4 * i + 2], p[4 * i + 3]);
}

__device__ __forceinline__ void load_planes16(const uint32_t* __restrict__ planes, int64_t g, uint32_t* p) {
  const uint4* q = reinterpret_cast<const uint4*>(planes + g * kPW16);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint4 v = q[i];
    p[4 * i] = v.x;
    p[4 * i + 1] = v.y;
    p[4 * i + 2] = v.z;
    p[4 * i + 3] = v.w;
  }
}

// ---------------------------------------------------------------- seed (int8)
// buf[(z - z0) 2^16 + c] = m(c) - 2 sum over groups of popc(XOR of the planes of z's bits), a
// workgroup = 256 columns x walks of 64 slices: the step-major walk of seed_sm_kernel in
// spectral.hip (per step every group's XOR and popcount, the sum straight into the byte stage;
// the first three groups' planes in registers, a fourth from L2), int8 byte staging and
// store-out as there.
template <int G>
__device__ __forceinline__ void walk_start16(const uint32_t (*pr)[kHi16], int zblk, uint32_t* x) {
#pragma unroll
  for (int g = 0; g < G; ++g) {
    uint32_t v = 0;
#pragma unroll
    for (int k = kWalkBits16; k < kHi16; ++k)
      if ((zblk >> k) & 1) v ^= pr[g][k];
    x[g] = v;
  }
}

// 64 Gray steps from the start state x, which is left at the last slice's state (plane 5 flipped)
template <int G>
__device__ __forceinline__ void walk_from16(const uint32_t (*pr)[kHi16], uint32_t* x, uint8_t* st8, int tid) {
#pragma unroll
  for (int i = 0; i < kWalk16; ++i) {
    uint32_t a = 0;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (i) x[g] ^= pr[g][ctz_c(i)];
      a = g ? popc_add(x[g], a) : (uint32_t)__popc(x[g]);  // one v_bcnt per group, no v_add3
    }
    st8[gray(i) * 256 + tid] = (uint8_t)a;
    if ((i & 7) == 7) __builtin_amdgcn_sched_barrier(0);
  }
}

constexpr int kRegGroups16 = 3;           // groups whose planes stay in registers
constexpr int kMaxWalkBlockBits16 = 4;    // walks per Gray-ordered block: <= 16

// after the register groups' walk of slices zblk..zblk + 63: the groups past them from L2, then
// the stage to HBM
__device__ __forceinline__ void seed16_finish(const uint32_t* __restrict__ planes, uint32_t g0, int ng, int wng,
                                              uint8_t* st8, int tid, int co, const uint32_t* mx, int mcb, int c0,
                                              int zblk, int z0, int z1, int8_t* __restrict__ buf) {
  constexpr int NT = 256;
  for (int g = kRegGroups16; g < wng; ++g) {  // the groups past the register-resident ones, from L2
    uint32_t p[kHi16];
    if (g < ng) {
      load_planes16(planes, (int64_t)g0 + g, p);
    } else {
#pragma unroll
      for (int k = 0; k < kHi16; ++k) p[k] = 0u;
    }
    uint32_t x = 0;
#pragma unroll
    for (int k = kWalkBits16; k < kHi16; ++k)
      if ((zblk >> k) & 1) x ^= p[k];
#pragma unroll
    for (int i = 0; i < kWalk16; ++i) {
      if (i) x ^= p[ctz_c(i)];
      st8[gray(i) * NT + co] += (uint8_t)__popc(x);
      if ((i & 7) == 7) __builtin_amdgcn_sched_barrier(0);
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kWalk16 / 16; ++r) {
    const int row = tid / (NT / 16) + 16 * r, z = zblk + row;
    const uint4 v = *reinterpret_cast<const uint4*>(st8 + row * NT + mcb);
    const uint4 o = make_uint4((mx[0] - (v.x + v.x)) ^ 0x80808080u, (mx[1] - (v.y + v.y)) ^ 0x80808080u,
                               (mx[2] - (v.z + v.z)) ^ 0x80808080u, (mx[3] - (v.w + v.w)) ^ 0x80808080u);
    if (z >= z0 && z < z1) *reinterpret_cast<uint4*>(buf + (int64_t)(z - z0) * kLo16 + c0 + mcb) = o;
  }
}

// the walks in Gray-ordered blocks of 2^lp, as seed_walks in spectral.hip
template <int G>
__device__ __forceinline__ void seed16_walks(const uint32_t (*pr)[kHi16], const uint32_t* __restrict__ planes,
                                             uint32_t g0, int ng, int wng, uint8_t* st8, int tid, int co,
                                             const uint32_t* mx, int mcb, int c0, int z0, int z1,
                                             int8_t* __restrict__ buf, int lp) {
  const int wa = (z0 & ~(kWalk16 - 1)) >> kWalkBits16, we = (z1 + kWalk16 - 1) >> kWalkBits16, P = 1 << lp;
  const int b1 = (we + P - 1) >> lp;
  for (int b = (wa >> lp) + blockIdx.y; b < b1; b += gridDim.y) {
    uint32_t x[G];
    walk_start16<G>(pr, (b << lp) << kWalkBits16, x);
    for (int j = 0; j < P; ++j) {  // workgroup-uniform
      if (j) {
        const int t = __builtin_ctz(j);
#pragma unroll
        for (int g = 0; g < G; ++g) {
          uint32_t f = pr[g][kWalkBits16 - 1];
#pragma unroll
          for (int k = 0; k < kMaxWalkBlockBits16; ++k)
            if (k == t) f ^= pr[g][kWalkBits16 + k];
          x[g] ^= f;
        }
      }
      const int w = (b << lp) + (j ^ (j >> 1));
      if (w < wa || w >= we) {  // outside the range: the state as if walked
#pragma unroll
        for (int g = 0; g < G; ++g) x[g] ^= pr[g][kWalkBits16 - 1];
        continue;
      }
      __syncthreads();  // the previous walk's store-out reads of `stage` are done
      walk_from16<G>(pr, x, st8, co);
      seed16_finish(planes, g0, ng, wng, st8, tid, co, mx, mcb, c0, w << kWalkBits16, z0, z1, buf);
    }
  }
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5))) void seed16_sm_kernel(
    const uint32_t* __restrict__ planes, const uint32_t* __restrict__ gofs, const uint32_t* __restrict__ off, int z0,
    int z1, int8_t* __restrict__ buf, int lp) {
  constexpr int NT = 256;
  __shared__ uint32_t stage[kWalk16 * NT / 4];
  uint8_t* st8 = reinterpret_cast<uint8_t*>(stage);
  const int tid = threadIdx.x;
  const int c0 = blockIdx.x * NT;
  // columns to lanes by group count (seed_lane_column, spectral.h): at config 5's density 1 in 8
  // columns holds more than 64 codes, so in column order nearly every wave walks 3 groups
  const int co = seed_lane_column(gofs, c0, tid);
  const int c = c0 + co;
  const uint32_t g0 = gofs[c];
  const int ng = (int)(gofs[c + 1] - g0);
  int wng = ng;
#pragma unroll
  for (int s = 32; s; s >>= 1) wng = max(wng, __shfl_xor(wng, s));
  uint32_t pr[kRegGroups16][kHi16];
#pragma unroll
  for (int g = 0; g < kRegGroups16; ++g)
    if (g < ng) {
      load_planes16(planes, (int64_t)g0 + g, pr[g]);
    } else {
#pragma unroll
      for (int k = 0; k < kHi16; ++k) pr[g][k] = 0u;
    }
  const int mcb = (tid % (NT / 16)) * 16;
  uint32_t mx[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    mx[k] = 0x80808080u;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int cc = c0 + mcb + 4 * k + b;
      mx[k] |= (off[cc + 1] - off[cc]) << (8 * b);
    }
  }
  {
    const int ph = (blockIdx.x + blockIdx.y) % 3;
    if (ph >= 1) __builtin_amdgcn_s_sleep(24);
    if (ph == 2) __builtin_amdgcn_s_sleep(24);
  }
  if (wng <= 1) seed16_walks<1>(pr, planes, g0, ng, wng, st8, tid, co, mx, mcb, c0, z0, z1, buf, lp);
  else if (wng == 2) seed16_walks<2>(pr, planes, g0, ng, wng, st8, tid, co, mx, mcb, c0, z0, z1, buf, lp);
  else seed16_walks<3>(pr, planes, g0, ng, wng, st8, tid, co, mx, mcb, c0, z0, z1, buf, lp);
}

// ---------------------------------------------------------------- tile
typedef int v4i_t __attribute__((ext_vector_type(4)));
typedef long v2l_t __attribute__((ext_vector_type(2)));
typedef short v2s_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ v2l_t pack16(const uint32_t* w) {
  return v2l_t{(long)(((uint64_t)w[1] << 32) | w[0]), (long)(((uint64_t)w[3] << 32) | w[2])};
}
__device__ __forceinline__ uint32_t pk_add16(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_bit_cast(v2s_t, a) + __builtin_bit_cast(v2s_t, b));
}

// LDS image of U_r: 64-bit word ((r * 4 + q) * 4 + mt) * 64 + lane holds the two int16 pairs
// (h = 0, 1) of stage-1 outputs of quarter q, load mt, lane -- the pairs16 layout of
// spectral.hip -- so one ds_add_u64 / ds_read_b64 moves four values (no half ever carries, so
// neither does the low dword)
constexpr int kUWords = 4 * 4 * 4 * 64;

// Stage-1 outputs y = v + 8192 (MFMA accumulator start 8192, |v| <= 64 * 127): every y lies
// in [64, 16320], so the four waves' packed pairs add into one LDS word without a carry
// (<= 65280 per half), and the two-byte split of y gives 256 hi + lo = v + 8064, whose
// stage-2 transform exceeds H v by 64 * 8064 at Q' = 0 only -- the high-byte MFMA of the
// q2 = 0 tile starts from -2016 there (-2016 * 256 = -516096).
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void tile16_kernel(
    const int8_t* __restrict__ buf, const uint16_t* __restrict__ order, int z0, int nslices,
    unsigned long long* __restrict__ counts, unsigned long long add_n, const unsigned long long* __restrict__ sumsq) {
  // every 16-bit column holds <= 127 codes: sum_w S_w = 2^32 sum f^2 <= 2^32 * 2^16 * 127^2 < 2^62,
  // so the 64-bit register / LDS sums cannot wrap
  __shared__ unsigned long long U[kUWords];
  __shared__ unsigned long long bins[17];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;  // wave = S (column digit 7)
  if (tid < 17) bins[tid] = 0;
  for (int w = tid; w < kUWords; w += 256) U[w] = 0;
  __syncthreads();
  v2l_t H[4];  // H_64 rows 16 q + (l & 15), columns 16 (l >> 4) + j
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t w[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      uint32_t v = 0;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * q + (lane & 15), col = 16 * (lane >> 4) + 4 * d + r;
        v |= ((__popc(row & col) & 1) ? 0xFFu : 0x01u) << (8 * r);
      }
      w[d] = v;
    }
    H[q] = pack16(w);
  }
  const v4i_t corr = v4i_t{lane < 16 ? -2016 : 0, 0, 0, 0};  // Q' = 0: lanes 0-15, element 0 of q2 = 0
  const int wt_thread = digit_weight((uint32_t)(lane & 15)) + digit_weight((uint32_t)(lane >> 4));
  const int wt_q = digit_weight((uint32_t)wave);  // this wave's U / V quarter (P' bits 4, 5)
  const int lane_off = 16 * (lane >> 4) + 64 * (lane & 15) + 16384 * wave;
  const int ub = (int)((int64_t)nslices * blockIdx.x / gridDim.x);
  const int ue = (int)((int64_t)nslices * (blockIdx.x + 1) / gridDim.x);
  // own planes: accG = sum G^2, accT = T_s^2 (index: compile-time digit weight of (P', Q'));
  // quarter `wave` of U_r / V: accU, accV (index without the quarter's digit)
  unsigned long long accG[4] = {0, 0, 0, 0}, accT[4] = {0, 0, 0, 0}, accU[3] = {0, 0, 0}, accV[3] = {0, 0, 0};
  int cur_w = -1;
  auto flush = [&]() {
    const int b = cur_w + wt_thread;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (accT[k]) atomicAdd(&bins[b + k + 1], 4 * accT[k]);
      const unsigned long long two = 16 * accG[k] - 4 * accT[k];
      if (two) atomicAdd(&bins[b + k + 2], two);
      accG[k] = accT[k] = 0;
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int bq = b + wt_q + k;
      if (accV[k]) atomicAdd(&bins[bq], accV[k]);
      const unsigned long long one = 4 * accU[k] - 2 * accV[k], two = accV[k] - 4 * accU[k];
      if (one) atomicAdd(&bins[bq + 1], one);
      if (two) atomicAdd(&bins[bq + 2], two);
      accU[k] = accV[k] = 0;
    }
  };
  auto load_plane = [&](int sl, int R, v2l_t* dst) {
    const int8_t* p = buf + (int64_t)sl * kLo16 + lane_off + 4096 * R;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
      dst[mt] = __builtin_nontemporal_load(reinterpret_cast<const v2l_t*>(p + 1024 * mt));
  };
  // stage 2 of two byte-split inputs a, b (quarters of P' with compile-time weights wa, wb;
  // wa = wb = 0 when the quarter's weight is added at flush), squares into acc
  auto stage2x2 = [&](const v2l_t& Bla, const v2l_t& Bha, const v2l_t& Blb, const v2l_t& Bhb, auto wa_c, auto wb_c,
                      bool corrected, unsigned long long* acc) {
    constexpr int wa = decltype(wa_c)::value, wb = decltype(wb_c)::value;
    v4i_t ca[4], cb[4];
#pragma unroll
    for (int q2 = 0; q2 < 4; ++q2) {
      const v4i_t c0 = (q2 == 0 && corrected) ? corr : v4i_t{0, 0, 0, 0};
      ca[q2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(H[q2], Bha, c0, 0, 0, 0);
      cb[q2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(H[q2], Bhb, c0, 0, 0, 0);
    }
#pragma unroll
    for (int q2 = 0; q2 < 4; ++q2) {
#pragma unroll
      for (int i = 0; i < 4; ++i) ca[q2][i] <<= 8;
      ca[q2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(H[q2], Bla, ca[q2], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 4; ++i) cb[q2][i] <<= 8;
      cb[q2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(H[q2], Blb, cb[q2], 0, 0, 0);
    }
#pragma unroll
    for (int q2 = 0; q2 < 4; ++q2)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        acc[wa + digit_weight_c((uint32_t)q2) + digit_weight_c((uint32_t)i)] +=
            (unsigned long long)((int64_t)ca[q2][i] * ca[q2][i]);
        acc[wb + digit_weight_c((uint32_t)q2) + digit_weight_c((uint32_t)i)] +=
            (unsigned long long)((int64_t)cb[q2][i] * cb[q2][i]);
      }
  };
  auto split16 = [&](const uint32_t (*pr)[2], v2l_t& Bl, v2l_t& Bh) {
    uint32_t lo[4], hi[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      lo[mt] = __builtin_amdgcn_perm(pr[mt][1], pr[mt][0], 0x06040200u) ^ 0x80808080u;
      hi[mt] = __builtin_amdgcn_perm(pr[mt][1], pr[mt][0], 0x07050301u);
    }
    Bl = pack16(lo);
    Bh = pack16(hi);
  };
  auto pairs16 = [&](const v4i_t* c1, uint32_t (*pr)[2]) {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      pr[mt][0] = __builtin_amdgcn_perm((uint32_t)c1[mt][1], (uint32_t)c1[mt][0], 0x05040100u);
      pr[mt][1] = __builtin_amdgcn_perm((uint32_t)c1[mt][3], (uint32_t)c1[mt][2], 0x05040100u);
    }
  };
  for (int u = ub; u < ue; ++u) {
    const int s = order ? (int)order[u] : u;
    const int wz = digit_weight((uint32_t)(z0 + s));  // workgroup-uniform
    if (wz != cur_w) {
      if (cur_w >= 0) flush();
      cur_w = wz;
    }
    uint32_t csp[4][4][2];  // T_s: sum over r of y as int16 pairs, from -32640 (-> sum v + 128)
#pragma unroll
    for (int qn = 0; qn < 4; ++qn)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) csp[qn][mt][0] = csp[qn][mt][1] = 0x80808080u;
    v2l_t dn[4];
    load_plane(s, 0, dn);
#pragma unroll 1
    for (int R = 0; R < 4; ++R) {
      v2l_t d[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) d[mt] = dn[mt];
      if (R < 3) load_plane(s, R + 1, dn);
      unsigned long long* Ur = U + R * (4 * 4 * 64) + lane;
      auto quarters = [&](auto qa_c, auto qb_c) {
        constexpr int qa = decltype(qa_c)::value, qb = decltype(qb_c)::value;
        v4i_t c1a[4], c1b[4];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          c1a[mt] = __builtin_amdgcn_mfma_i32_16x16x64_i8(d[mt], H[qa], v4i_t{8192, 8192, 8192, 8192}, 0, 0, 0);
          c1b[mt] = __builtin_amdgcn_mfma_i32_16x16x64_i8(d[mt], H[qb], v4i_t{8192, 8192, 8192, 8192}, 0, 0, 0);
        }
        uint32_t pa[4][2], pb[4][2];
        pairs16(c1a, pa);
        pairs16(c1b, pb);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            csp[qa][mt][h] = pk_add16(csp[qa][mt][h], pa[mt][h]);
            csp[qb][mt][h] = pk_add16(csp[qb][mt][h], pb[mt][h]);
          }
          atomicAdd(Ur + (qa * 4 + mt) * 64, ((unsigned long long)pa[mt][1] << 32) | pa[mt][0]);
          atomicAdd(Ur + (qb * 4 + mt) * 64, ((unsigned long long)pb[mt][1] << 32) | pb[mt][0]);
        }
        v2l_t Bla, Bha, Blb, Bhb;
        split16(pa, Bla, Bha);
        split16(pb, Blb, Bhb);
        stage2x2(Bla, Bha, Blb, Bhb, std::integral_constant<int, digit_weight_c(qa)>(),
                 std::integral_constant<int, digit_weight_c(qb)>(), true, accG);
        __builtin_amdgcn_sched_barrier(0);
      };
      quarters(std::integral_constant<int, 0>(), std::integral_constant<int, 1>());
      quarters(std::integral_constant<int, 2>(), std::integral_constant<int, 3>());
    }
    {  // T_s = this wave's plane sum
      v2l_t Bla, Bha, Blb, Bhb;
      split16(csp[0], Bla, Bha);
      split16(csp[1], Blb, Bhb);
      stage2x2(Bla, Bha, Blb, Bhb, std::integral_constant<int, 0>(), std::integral_constant<int, 1>(), false, accT);
      split16(csp[2], Bla, Bha);
      split16(csp[3], Blb, Bhb);
      stage2x2(Bla, Bha, Blb, Bhb, std::integral_constant<int, 1>(), std::integral_constant<int, 1>(), false, accT);
    }
    __syncthreads();  // every wave's U adds are in
    {  // quarter q = wave of U_0..U_3; V = sum_r U_r from the sum of their stage-2 outputs
      uint32_t uu[4][4][2];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          unsigned long long* p = U + ((r * 4 + wave) * 4 + mt) * 64 + lane;
          const unsigned long long v = *p;
          *p = 0ull;  // read by this wave only: cleared for the next slice
          // + 0x8080 per half (mod 2^16) turns U + 32768 into U + 128 (the csp form)
          uu[r][mt][0] = pk_add16((uint32_t)v, 0x80808080u);
          uu[r][mt][1] = pk_add16((uint32_t)(v >> 32), 0x80808080u);
        }
      v4i_t fv[4] = {v4i_t{0, 0, 0, 0}, v4i_t{0, 0, 0, 0}, v4i_t{0, 0, 0, 0}, v4i_t{0, 0, 0, 0}};
#pragma unroll
      for (int r = 0; r < 4; r += 2) {
        v2l_t Bla, Bha, Blb, Bhb;
        split16(uu[r], Bla, Bha);
        split16(uu[r + 1], Blb, Bhb);
        v4i_t ca[4], cb[4];
#pragma unroll
        for (int q2 = 0; q2 < 4; ++q2) {
          ca[q2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(H[q2], Bha, v4i_t{0, 0, 0, 0}, 0, 0, 0);
          cb[q2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(H[q2], Bhb, v4i_t{0, 0, 0, 0}, 0, 0, 0);
        }
#pragma unroll
        for (int q2 = 0; q2 < 4; ++q2) {
#pragma unroll
          for (int i = 0; i < 4; ++i) ca[q2][i] <<= 8;
          ca[q2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(H[q2], Bla, ca[q2], 0, 0, 0);
#pragma unroll
          for (int i = 0; i < 4; ++i) cb[q2][i] <<= 8;
          cb[q2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(H[q2], Blb, cb[q2], 0, 0, 0);
        }
#pragma unroll
        for (int q2 = 0; q2 < 4; ++q2)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int k = digit_weight_c((uint32_t)q2) + digit_weight_c((uint32_t)i);
            accU[k] += (unsigned long long)((int64_t)ca[q2][i] * ca[q2][i]);
            accU[k] += (unsigned long long)((int64_t)cb[q2][i] * cb[q2][i]);
            fv[q2][i] += ca[q2][i] + cb[q2][i];  // |V's transform| <= 64 * 16 * 8128
          }
      }
#pragma unroll
      for (int q2 = 0; q2 < 4; ++q2)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          accV[digit_weight_c((uint32_t)q2) + digit_weight_c((uint32_t)i)] +=
              (unsigned long long)((int64_t)fv[q2][i] * fv[q2][i]);
    }
    __syncthreads();  // U cleared before the next slice's adds
  }
  if (cur_w >= 0) flush();
  __syncthreads();
  if (tid < 17) add_weight_sum64(counts, tid, bins[tid]);
  add_job_constants(counts, add_n, sumsq);
}

void launch_seed16(State& st, int8_t* buf, int z0, int z1, hipStream_t s) {
  const int walks = (z1 - (z0 & ~(kWalk16 - 1)) + kWalk16 - 1) / kWalk16;
  const int per_wg = std::max(1, std::min(kSeedWalks16, walks / 16));
  int lp = 0;  // walks per Gray-ordered block: the largest power of two <= per_wg, <= 16
  while (lp < kMaxWalkBlockBits16 && (2 << lp) <= per_wg) ++lp;
  const int wa = (z0 & ~(kWalk16 - 1)) / kWalk16, we = (z1 + kWalk16 - 1) / kWalk16;
  const int nb = ((we + (1 << lp) - 1) >> lp) - (wa >> lp);
  hipLaunchKernelGGL(seed16_sm_kernel, dim3(kLo16 / 256, (unsigned)nb), dim3(256), 0, s, st.d_planes, st.d_gofs, st.d_off,
                     z0, z1, buf, lp);
}

void launch_tile16(State& st, const int8_t* buf, int z0, int z1, unsigned long long* counts, hipStream_t s,
                   unsigned long long add_n, int wgs_per_cu) {
  const int ns = z1 - z0;
  const uint16_t* order = ((ns & (ns - 1)) == 0 && ns <= (1 << 16) && z0 % ns == 0) ? st.d_order + ns : nullptr;
  hipLaunchKernelGGL(tile16_kernel, dim3((unsigned)std::max(1, std::min(st.grid * wgs_per_cu, ns))), dim3(256), 0, s,
                     buf, order, z0, ns, counts, add_n, st.sumsq_ptr());
}

int launch_chunk16(State& st, int z0, int z1, unsigned long long* counts, hipStream_t s, unsigned long long add_n) {
  int8_t* buf = reinterpret_cast<int8_t*>(st.d_buf);
  hipEvent_t t0 = st.timer ? st.timer->start(s) : nullptr;
  launch_seed16(st, buf, z0, z1, s);
  SCT_LAUNCH_CHECK();
  if (st.timer) st.timer->stop(s, t0, sct::LaunchTimer::SEED);
  t0 = st.timer ? st.timer->start(s) : nullptr;
  launch_tile16(st, buf, z0, z1, counts, s, add_n, st.tile_wgs);
  SCT_LAUNCH_CHECK();
  if (st.timer) st.timer->stop(s, t0, sct::LaunchTimer::TILE);
  return SCT_OK;
}

// virtual slices [b, e) of 2^18 -> real 16-bit slices [ceil(b / 4), ceil(e / 4)): a partition of
// the virtual range maps to a partition of the real one
inline int64_t real16(int64_t z) { return (z + 3) >> 2; }

}  // namespace

int create16(State& st, const uint64_t* d_codes, int64_t n, unsigned max16, int64_t chunk, int cus) {
  st.lo_bits = kLoBits16;
  st.max_m = max16;
  st.elem_bytes = 1;
  st.chunk16 = std::max<int64_t>(kWalk16, std::min<int64_t>(kChunk16, chunk / 4));
  st.chunk = 4 * st.chunk16;  // in virtual slices (the plan's items)
  static const int per_cu = [] {
    int v = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, tile16_kernel, 256, 0) != hipSuccess || v <= 0) v = 2;
    return v;
  }();
  st.tile_wgs = per_cu;
  if (int rc = make_order_table(st); rc != SCT_OK) return rc;
  st.max_groups = sct::ceil_div(n, 32) + kLo16;
  void* p = nullptr;
  auto get = [&](int slot, size_t bytes, auto** out) {
    const int rc = ws_get(st.ws, slot, bytes, &p);
    if (rc == SCT_OK) *out = reinterpret_cast<std::remove_reference_t<decltype(**out)>*>(p);
    return rc;
  };
  if (int rc = get(W_HI, (size_t)n * 4, &st.d_hi); rc != SCT_OK) return rc;
  if (int rc = get(W_OFF, (size_t)(kLo16 + 1) * 4, &st.d_off); rc != SCT_OK) return rc;
  if (int rc = get(W_CNT, (size_t)kLo16 * 4, &st.d_cnt); rc != SCT_OK) return rc;
  if (int rc = get(W_GOFS, (size_t)(kLo16 + 1) * 4, &st.d_gofs); rc != SCT_OK) return rc;
  if (int rc = get(W_HIST, (size_t)kSortWGs16 * kLo16, &st.d_hist); rc != SCT_OK) return rc;
  if (int rc = get(W_PLANES, (size_t)st.max_groups * kPW16 * 4, &st.d_planes); rc != SCT_OK) return rc;
  if (int rc = alloc_buf(st, &st.chunk16, std::min<int64_t>(st.chunk16, 1024), (size_t)kLo16); rc != SCT_OK) return rc;
  st.chunk = 4 * st.chunk16;
  if (int rc = get(W_SUMSQ, sizeof(unsigned long long), &st.d_sumsq); rc != SCT_OK) return rc;
  return SCT_OK;
}

int build16(State& st, const uint64_t* d_codes, hipStream_t s) {
  hipEvent_t t0 = st.timer ? st.timer->start(s) : nullptr;
  hipLaunchKernelGGL(hist16_wg_kernel, dim3(kSortWGs16), dim3(kSortThreads16), 0, s, d_codes, st.n, st.d_hist);
  SCT_LAUNCH_CHECK();
  hipLaunchKernelGGL(prefix16_kernel, dim3(kLo16 / 4 / 256), dim3(256), 0, s, st.d_hist, kSortWGs16, st.d_cnt);
  SCT_LAUNCH_CHECK();
  hipLaunchKernelGGL(scan16_kernel, dim3(1), dim3(1024), 0, s, st.d_cnt, st.d_off, st.d_gofs);
  SCT_LAUNCH_CHECK();
  hipLaunchKernelGGL(scatter16_wg_kernel, dim3(kSortWGs16), dim3(kSortThreads16), 0, s, d_codes, st.n, st.d_hist,
                     st.d_off, st.d_hi);
  SCT_LAUNCH_CHECK();
  hipLaunchKernelGGL(planes16_kernel, dim3(kLo16 * 4 / 256), dim3(256), 0, s, st.d_hi, st.d_off, st.d_gofs,
                     st.d_planes);
  SCT_LAUNCH_CHECK();
  if (st.timer) st.timer->stop(s, t0, sct::LaunchTimer::BUILD);
  return SCT_OK;
}

int count16(State& st, int64_t z_begin, int64_t z_end, unsigned long long* d_counts, hipStream_t s) {
  const int64_t rb = real16(z_begin), re = real16(z_end);
  for (int64_t z0 = rb; z0 < re; z0 += st.chunk16) {
    const int z1 = (int)std::min<int64_t>(re, z0 + st.chunk16);
    const unsigned long long add_n = z0 == 0 ? (unsigned long long)st.n : 0ull;
    if (int rc = launch_chunk16(st, (int)z0, z1, d_counts, s, add_n); rc != SCT_OK) return rc;
  }
  return SCT_OK;
}

int time_kernels16(State& st, int64_t z_begin, int64_t z_end, unsigned long long* d_counts, int repeats,
                   hipStream_t s, double* seed_ms, double* tile_ms, int64_t* slices) {
  const int64_t rb = real16(z_begin), re = std::min<int64_t>(real16(z_end), rb + st.chunk16);
  SCT_CHECK(rb < re, "time_kernels: empty 16-bit slice range");
  *slices = 4 * (re - rb);  // virtual slices (the bench prices 16 KiB per virtual slice)
  hipEvent_t e[3];
  for (auto& x : e) SCT_HIP(hipEventCreate(&x));
  struct Free {
    hipEvent_t* e;
    ~Free() {
      for (int i = 0; i < 3; ++i) (void)hipEventDestroy(e[i]);
    }
  } guard{e};
  sct::LaunchTimer* keep = st.timer;
  st.timer = nullptr;
  int rc = launch_chunk16(st, (int)rb, (int)re, d_counts, s, 0);  // warm
  int8_t* buf = reinterpret_cast<int8_t*>(st.d_buf);
  const int ns = (int)(re - rb);
  const uint16_t* order = ((ns & (ns - 1)) == 0 && ns <= (1 << 16) && rb % ns == 0) ? st.d_order + ns : nullptr;
  SCT_HIP(hipEventRecord(e[0], s));
  for (int r = 0; rc == SCT_OK && r < repeats; ++r) launch_seed16(st, buf, (int)rb, (int)re, s);
  SCT_HIP(hipEventRecord(e[1], s));
  for (int r = 0; rc == SCT_OK && r < repeats; ++r)
    hipLaunchKernelGGL(tile16_kernel, dim3((unsigned)std::max(1, std::min(st.grid * st.tile_wgs, ns))), dim3(256), 0,
                       s, buf, order, (int)rb, ns, d_counts, 0ull, st.sumsq_ptr());
  SCT_HIP(hipEventRecord(e[2], s));
  st.timer = keep;
  if (rc != SCT_OK) return rc;
  SCT_HIP(hipEventSynchronize(e[2]));
  float a = 0, b = 0;
  SCT_HIP(hipEventElapsedTime(&a, e[0], e[1]));
  SCT_HIP(hipEventElapsedTime(&b, e[1], e[2]));
  *seed_ms = a / repeats;
  *tile_ms = b / repeats;
  return SCT_OK;
}

}  // namespace sct_spectral
