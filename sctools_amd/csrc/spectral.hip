// Spectral all-pairs scheme: the TwoBit distance histogram of n 16-base codes from the
// Walsh-Hadamard transform of their multiplicity f over Z_2^32.
//
//   d(x, y) = digit weight of x ^ y (non-zero 2-bit digits), so the ordered-pair counts
//   N(d) = sum_{v : wt(v) = d} R(v), R = f (*) f (XOR autocorrelation), and with
//   F = WHT(f):  N(d) = 2^-32 sum_z F(z)^2 K_d(wt(z)),  K_d the q = 4 Krawtchouk
//   polynomial.  The device computes S_w = sum_{wt(z) = w} F(z)^2 (17 uint64); the host
//   (sct_counts_to_hist_ex) applies K and halves: hist[d] = (N(d) - n [d = 0]) / 2.
//
// z = (slice z >> 14, column z & 0x3FFF); the 2^18 slices are the plan's work items.
//   seed   F's partial sums over the high 18 bits, per column, from bit planes of the
//          column's codes: a Gray-code walk over 64 slices costs one XOR and one
//          popcount per 32 codes per value.  |seed| <= codes in the column, so the
//          values go to HBM as int8 (int16 / int32 for denser columns): 16 KB per slice
//   tile   reads a slice back, transforms it over the 14 column bits (int8 seeds: two
//          64-point stages on the matrix cores + Parseval for the top digit), F^2 binned
//          by digit weight; writes nothing
// 8 GB of HBM traffic per job at int8, whatever n is.  Exact: |F| <= n <= 1e8 in int32,
// F^2 in uint64, S_w in three non-carrying limbs (spectral.h: sum_w S_w = 2^32 sum f^2 exceeds
// 2^64 for multisets with sum f^2 >= 2^32).
#include <string.h>

#include <algorithm>
#include <vector>
#include <type_traits>

#include <mutex>

#include <hipcub/hipcub.hpp>

#include "sct_common.h"
#include "spectral.h"

namespace sct_spectral {
namespace {

constexpr int kLo = 1 << kLoBits;         // columns (= tile values)
constexpr int kHiBits = kSpaceBits - kLoBits;  // 18 bit planes
constexpr int kWalk = 64;                 // slices per wave in the seed's Gray walk
constexpr int kWalkBits = 6;
constexpr int kRegGroups = 2;             // seed: 32-code groups whose planes stay in registers
constexpr int kSeedWalks = 16;            // seed: walks per workgroup (4-32 within noise, round 3)
constexpr int kMaxOrder = 1 << 16;        // largest slice range with a digit-weight order table

// Bit planes of a 32-code group: planes + g * kPlaneWords holds its 18 planes (plane k bit j =
// bit k of (code >> 14) of the group's j-th code) and 2 words of padding, so a group's planes
// are five aligned 16-B words: one lane's group is 5 loads from 2 lines, not 18 from 18.
constexpr int kPlaneWords = 20;
__device__ __forceinline__ void load_planes(const uint32_t* __restrict__ planes, int64_t g, uint32_t* p) {
  const uint4* q = reinterpret_cast<const uint4*>(planes + g * kPlaneWords);
  uint32_t w[kPlaneWords];
#pragma unroll
  for (int i = 0; i < kPlaneWords / 4; ++i) {
    const uint4 v = q[i];
    w[4 * i] = v.x;
    w[4 * i + 1] = v.y;
    w[4 * i + 2] = v.z;
    w[4 * i + 3] = v.w;
  }
#pragma unroll
  for (int k = 0; k < 18; ++k) p[k] = w[k];
}
__device__ __forceinline__ void store_planes(uint32_t* __restrict__ planes, int64_t g, const uint32_t* p) {
  uint4* q = reinterpret_cast<uint4*>(planes + g * kPlaneWords);
#pragma unroll
  for (int i = 0; i < kPlaneWords / 4; ++i)
    q[i] = make_uint4(4 * i < 18 ? p[4 * i] : 0u, 4 * i + 1 < 18 ? p[4 * i + 1] : 0u,
                      4 * i + 2 < 18 ? p[4 * i + 2] : 0u, 4 * i + 3 < 18 ? p[4 * i + 3] : 0u);
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

// Privatised counting sort (the build of every step; no global atomics):
//   hist_wg   workgroup g counts its contiguous share of the codes per column in LDS and
//             writes the 2^14 counts to H[g][.]
//   prefix    per column: H[g][c] <- sum of H[g' < g][c] (in place), m(c) = the total
//   scan      one workgroup: off / gofs = exclusive scans of m(c) and ceil(m(c) / 32)
//   scatter   workgroup g: LDS cursors off[c] + H[g][c], one LDS atomic per code
constexpr int kSortWGs = 128;
constexpr int kSortThreads = 1024;

__device__ __forceinline__ void wg_range(int64_t n, int64_t& b, int64_t& e) {
  b = n * blockIdx.x / gridDim.x;
  e = n * (blockIdx.x + 1) / gridDim.x;
}

__global__ __launch_bounds__(kSortThreads) void column_hist_wg_kernel(const uint64_t* __restrict__ codes, int64_t n,
                                                                      uint32_t* __restrict__ H) {
  __shared__ uint32_t h[kLo];
  for (int c = threadIdx.x; c < kLo; c += kSortThreads) h[c] = 0;
  __syncthreads();
  int64_t b, e;
  wg_range(n, b, e);
  for (int64_t i = b + threadIdx.x; i < e; i += kSortThreads) atomicAdd(&h[codes[i] & (kLo - 1)], 1u);
  __syncthreads();
  uint32_t* out = H + (int64_t)blockIdx.x * kLo;
  for (int c = threadIdx.x; c < kLo; c += kSortThreads) out[c] = h[c];
}

__global__ __launch_bounds__(256) void column_prefix_kernel(uint32_t* __restrict__ H, int wgs,
                                                            uint32_t* __restrict__ m) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  uint32_t run = 0;
#pragma unroll 8
  for (int g = 0; g < wgs; ++g) {
    const uint32_t v = H[(int64_t)g * kLo + c];
    H[(int64_t)g * kLo + c] = run;
    run += v;
  }
  m[c] = run;
}

// one workgroup of 1024: 16 columns per thread, wave scans + one LDS pass over the waves
__global__ __launch_bounds__(1024) void column_scan16_kernel(const uint32_t* __restrict__ m,
                                                             uint32_t* __restrict__ off,
                                                             uint32_t* __restrict__ gofs) {
  __shared__ uint32_t wsum[2][16];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  uint32_t v[16];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint4 q = reinterpret_cast<const uint4*>(m)[t * 4 + k];
    v[4 * k] = q.x;
    v[4 * k + 1] = q.y;
    v[4 * k + 2] = q.z;
    v[4 * k + 3] = q.w;
  }
  uint32_t s = 0, sg = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    s += v[k];
    sg += (v[k] + 31) / 32;
  }
  uint32_t is = s, isg = sg;  // inclusive scans over the wave
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
  uint32_t base = 0, baseg = 0;
  for (int w = 0; w < wave; ++w) {
    base += wsum[0][w];
    baseg += wsum[1][w];
  }
  uint32_t run = base + is - s, rung = baseg + isg - sg;
  uint32_t o[16], og[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    o[k] = run;
    og[k] = rung;
    run += v[k];
    rung += (v[k] + 31) / 32;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    reinterpret_cast<uint4*>(off)[t * 4 + k] = make_uint4(o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]);
    reinterpret_cast<uint4*>(gofs)[t * 4 + k] = make_uint4(og[4 * k], og[4 * k + 1], og[4 * k + 2], og[4 * k + 3]);
  }
  if (t == 1023) {
    off[kLo] = run;
    gofs[kLo] = rung;
  }
}

__global__ __launch_bounds__(kSortThreads) void column_scatter_wg_kernel(const uint64_t* __restrict__ codes,
                                                                         int64_t n,
                                                                         const uint32_t* __restrict__ H,
                                                                         const uint32_t* __restrict__ off,
                                                                         uint32_t* __restrict__ hi) {
  __shared__ uint32_t cur[kLo];
  const uint32_t* pre = H + (int64_t)blockIdx.x * kLo;
  for (int c = threadIdx.x; c < kLo; c += kSortThreads) cur[c] = off[c] + pre[c];
  __syncthreads();
  int64_t b, e;
  wg_range(n, b, e);
  for (int64_t i = b + threadIdx.x; i < e; i += kSortThreads) {
    const uint64_t x = codes[i];
    hi[atomicAdd(&cur[x & (kLo - 1)], 1u)] = (uint32_t)(x >> kLoBits);
  }
}

// planes of group slot k of column c (thread (c, k); columns of <= 32 * kSlots codes)
template <int kSlots>
__global__ __launch_bounds__(256) void planes_slot_kernel(const uint32_t* __restrict__ hi,
                                                          const uint32_t* __restrict__ off,
                                                          const uint32_t* __restrict__ gofs, int64_t max_groups,
                                                          uint32_t* __restrict__ planes) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int c = t / kSlots, k = t % kSlots;
  const uint32_t g0 = gofs[c];
  if (k >= (int)(gofs[c + 1] - g0)) return;
  const uint32_t first = off[c] + 32u * k, last = min(first + 32u, off[c + 1]);
  uint32_t p[kHiBits];
#pragma unroll
  for (int b = 0; b < kHiBits; ++b) p[b] = 0;
  for (uint32_t i = first; i < last; ++i) {
    const uint32_t h = hi[i], bit = 1u << (i - first);
#pragma unroll
    for (int b = 0; b < kHiBits; ++b) p[b] |= (h >> b) & 1u ? bit : 0u;
  }
  const int64_t g = g0 + k;
  store_planes(planes, g, p);
}

// group g's planes (load_planes layout)
__global__ void planes_kernel(const uint32_t* __restrict__ hi, const uint32_t* __restrict__ off,
                              const uint32_t* __restrict__ gofs, int64_t max_groups,
                              uint32_t* __restrict__ planes) {
  const int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (g >= (int64_t)gofs[kLo]) return;
  int a = 0, b = kLo;  // column c: gofs[c] <= g < gofs[c + 1]
  while (b - a > 1) {
    const int m = (a + b) >> 1;
    if (gofs[m] <= (uint32_t)g) a = m;
    else b = m;
  }
  const uint32_t first = off[a] + 32u * ((uint32_t)g - gofs[a]);
  const uint32_t last = min(first + 32u, off[a + 1]);
  uint32_t p[kHiBits];
#pragma unroll
  for (int k = 0; k < kHiBits; ++k) p[k] = 0;
  for (uint32_t i = first; i < last; ++i) {
    const uint32_t h = hi[i], bit = 1u << (i - first);
#pragma unroll
    for (int k = 0; k < kHiBits; ++k) p[k] |= (h >> k) & 1u ? bit : 0u;
  }
  store_planes(planes, g, p);
}

typedef unsigned v4u __attribute__((ext_vector_type(4)));

// Value type of the seed -> tile intermediate: |seed| <= codes in the column, so the
// densest column decides (int8 for whitelists up to ~1.2M random barcodes).
template <typename T>
struct Chunk {
  static constexpr int kVals = 16 / sizeof(T);                  // columns per 16-B chunk
  static constexpr int kLog = sizeof(T) == 1 ? 4 : (sizeof(T) == 2 ? 3 : 2);
  static constexpr int kPerThread = 64 / kVals;                 // chunks per tile thread
};

// Position of column c inside a slice row of the intermediate.  Chosen so that the tile
// kernel's thread t, reading 16-B chunks at t*kVals + j*2^(kLog+8), receives the columns
// with bits 4..11 = t and registers q = column bits 0..3 + 16 * bits 12, 13, whatever T is.
template <typename T>
__device__ __forceinline__ int column_pos(int c) {
  constexpr int L = Chunk<T>::kLog;
  return (c & ((1 << L) - 1)) | (((c >> 4) & 255) << L) | (((c >> L) & ((16 >> L) - 1)) << (L + 8)) |
         ((c >> 12) << 12);
}


// int16 / int32 seeds (columns of more than 127 codes): a workgroup owns 256 columns and walks of
// 64 slices (blockIdx.y, strided): each lane walks its column in Gray order (one XOR per step
// from registers) group by group into a 64-value accumulator array; dwords of 4 / sizeof(T)
// consecutive slices per column are staged in LDS, transposed in registers and written as 16-B
// chunks of slice rows.  (int8 seeds: seed_sm_kernel below.)
template <typename T>
__device__ __forceinline__ void seed_body(const uint32_t* __restrict__ planes, const uint32_t* __restrict__ gofs,
                                          const uint32_t* __restrict__ off, int z0, int z1, T* __restrict__ buf) {
  constexpr int NT = 256;
  constexpr int P = 4 / sizeof(T);          // slices per staged dword
  constexpr int V = Chunk<T>::kVals;        // columns per 16-B output chunk
  __shared__ uint32_t stage[(kWalk / P) * NT];
  const int tid = threadIdx.x;
  const int c0 = blockIdx.x * NT, c = c0 + tid;
  const int m = (int)(off[c + 1] - off[c]);
  const uint32_t g0 = gofs[c];
  const int ng = (int)(gofs[c + 1] - g0);
  int wng = ng;
#pragma unroll
  for (int s = 32; s; s >>= 1) wng = max(wng, __shfl_xor(wng, s));
  // the first kRegGroups groups' planes stay in registers for all of this workgroup's walks
  uint32_t pr[kRegGroups][kHiBits];
#pragma unroll
  for (int g = 0; g < kRegGroups; ++g)
    if (g < ng) {
      load_planes(planes, (int64_t)g0 + g, pr[g]);
    } else {
#pragma unroll
      for (int k = 0; k < kHiBits; ++k) pr[g][k] = 0u;
    }
  // Co-resident workgroups start together and run identical walks, so they stay in
  // lockstep: all 12 waves of a CU walk (VALU-bound) and then all store (HBM-bound).
  // Starting them 0 / 1,536 / 3,072 cycles apart lets one workgroup's stores drain under
  // another's walk (What was tried (14)).
  {
    const int ph = (blockIdx.x + blockIdx.y) % 3;
    if (ph >= 1) __builtin_amdgcn_s_sleep(24);
    if (ph == 2) __builtin_amdgcn_s_sleep(24);
  }
  const int za = z0 & ~(kWalk - 1);
  const int nwalks = (z1 - za + kWalk - 1) / kWalk;
  for (int wk = blockIdx.y; wk < nwalks; wk += gridDim.y) {
    const int zblk = za + wk * kWalk;
    int acc[kWalk];
    auto walk = [&](const uint32_t* p, auto first) {
      uint32_t x = 0;
#pragma unroll
      for (int k = kWalkBits; k < kHiBits; ++k)
        if ((zblk >> k) & 1) x ^= p[k];
      if constexpr (decltype(first)::value) acc[0] = __popc(x);
      else acc[0] += __popc(x);
#pragma unroll
      for (int i = 1; i < kWalk; ++i) {
        x ^= p[ctz_c(i)];
        if constexpr (decltype(first)::value) acc[gray(i)] = __popc(x);
        else acc[gray(i)] += __popc(x);
      }
    };
    walk(pr[0], std::true_type());  // columns without codes: planes 0, popc 0
#pragma unroll
    for (int g = 1; g < kRegGroups; ++g)
      if (g < wng) walk(pr[g], std::false_type());
    for (int g = kRegGroups; g < wng; ++g) {  // dense columns: the rest from L2
      uint32_t p[kHiBits];
      if (g < ng) {
        load_planes(planes, (int64_t)g0 + g, p);
      } else {
#pragma unroll
        for (int k = 0; k < kHiBits; ++k) p[k] = 0u;
      }
      walk(p, std::false_type());
    }
    {
      __syncthreads();  // the previous walk's store-out reads of `stage` are done
      // 4-dword groups of a 16-dword column block XOR-swizzled by the block, so the
      // store-out's b128 reads of 16 consecutive columns are conflict-free
      auto sidx = [](int row, int col) { return row * 256 + (col ^ (((col >> 6) & 3) << 2)); };
#pragma unroll
      for (int r = 0; r < kWalk / P; ++r) {
        uint32_t w = 0;
#pragma unroll
        for (int j = 0; j < P; ++j)
          w |= ((uint32_t)(m - 2 * acc[r * P + j]) & (0xFFFFFFFFu >> (32 - 8 * sizeof(T)))) << (8 * sizeof(T) * j);
        stage[sidx(r, tid)] = w;
      }
      __syncthreads();
      // blocks of V columns x P slices: V dwords in, P chunks out
      constexpr int kBlocks = (kWalk / P) * (256 / V);
#pragma unroll
      for (int r = 0; r < kBlocks / 256; ++r) {
        const int b = tid + 256 * r, row = b / (256 / V), cb = (b % (256 / V)) * V;
        uint32_t d[V];
#pragma unroll
        for (int k = 0; k < V; k += 4) {
          const uint4 v = *reinterpret_cast<const uint4*>(stage + sidx(row, cb + k));
          d[k] = v.x;
          d[k + 1] = v.y;
          d[k + 2] = v.z;
          d[k + 3] = v.w;
        }
        uint32_t out[P][4];
        if constexpr (P == 2) {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            out[0][k] = __builtin_amdgcn_perm(d[2 * k + 1], d[2 * k], 0x05040100u);
            out[1][k] = __builtin_amdgcn_perm(d[2 * k + 1], d[2 * k], 0x07060302u);
          }
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k) out[0][k] = d[k];
        }
#pragma unroll
        for (int j = 0; j < P; ++j) {
          const int z = zblk + row * P + j;
          if (z < z0 || z >= z1) continue;
          *reinterpret_cast<uint4*>(buf + (int64_t)(z - z0) * kLo + column_pos<T>(c0 + cb)) =
              make_uint4(out[j][0], out[j][1], out[j][2], out[j][3]);
        }
      }
    }
  }
}

// int8 seeds, step-major walk: per step every group's XOR and popcount, and the step's sum
// goes to the byte stage at once -- no 64-value accumulator array, so the first three groups'
// planes stay in registers at 4+ waves per SIMD.  G = the wave's group count (<= 3; a fourth
// and later group, columns of > 96 codes, is walked afterwards from L2 into the lane's own
// stage bytes).  Store-out as seed_body<int8_t>.
// the walk's start state: every group's planes XORed for the slice bits 6..17 of zblk
template <int G>
__device__ __forceinline__ void walk_start(const uint32_t (*pr)[kHiBits], int zblk, uint32_t* x) {
#pragma unroll
  for (int g = 0; g < G; ++g) {
    uint32_t v = 0;
#pragma unroll
    for (int k = kWalkBits; k < kHiBits; ++k)
      if ((zblk >> k) & 1) v ^= pr[g][k];
    x[g] = v;
  }
}

// 64 Gray steps from the start state x; x is left at the last slice's state, which is the
// start state with plane 5 flipped (gray(63) = 32)
template <int G>
__device__ __forceinline__ void walk_from(const uint32_t (*pr)[kHiBits], uint32_t* x, uint8_t* st8, int tid) {
#pragma unroll
  for (int i = 0; i < kWalk; ++i) {
    uint32_t a = 0;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (i) x[g] ^= pr[g][ctz_c(i)];
      a = g ? popc_add(x[g], a) : (uint32_t)__popc(x[g]);  // one v_bcnt per group, no v_add3
    }
    st8[gray(i) * 256 + tid] = (uint8_t)a;
    if ((i & 7) == 7) __builtin_amdgcn_sched_barrier(0);  // keep the scheduler from hoisting steps
  }
}

constexpr int kRegGroupsSM = 3;
constexpr int kMaxWalkBlockBits = 4;  // walks per Gray-ordered block: <= 16

// after the register groups' walk of slices zblk..zblk + 63: the groups beyond them (columns of
// > 96 codes) from L2 into the lane's stage bytes, then the stage to HBM as int8 m - 2 * sum
__device__ __forceinline__ void seed_finish(const uint32_t* __restrict__ planes, uint32_t g0, int ng, int wng,
                                            uint8_t* st8, int tid, int co, const uint32_t* mx, int mcb, int c0,
                                            int zblk, int z0, int z1, int8_t* __restrict__ buf) {
  constexpr int NT = 256;
  for (int g = kRegGroupsSM; g < wng; ++g) {
    uint32_t p[kHiBits];
    if (g < ng) {
      load_planes(planes, (int64_t)g0 + g, p);
    } else {
#pragma unroll
      for (int k = 0; k < kHiBits; ++k) p[k] = 0u;
    }
    uint32_t x = 0;
#pragma unroll
    for (int k = kWalkBits; k < kHiBits; ++k)
      if ((zblk >> k) & 1) x ^= p[k];
#pragma unroll
    for (int i = 0; i < kWalk; ++i) {
      if (i) x ^= p[ctz_c(i)];
      st8[gray(i) * NT + co] += (uint8_t)__popc(x);
      if ((i & 7) == 7) __builtin_amdgcn_sched_barrier(0);
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kWalk / 16; ++r) {
    const int row = tid / (NT / 16) + 16 * r, z = zblk + row;
    const uint4 v = *reinterpret_cast<const uint4*>(st8 + row * NT + mcb);
    const uint4 o = make_uint4((mx[0] - (v.x + v.x)) ^ 0x80808080u, (mx[1] - (v.y + v.y)) ^ 0x80808080u,
                               (mx[2] - (v.z + v.z)) ^ 0x80808080u, (mx[3] - (v.w + v.w)) ^ 0x80808080u);
    if (z >= z0 && z < z1) *reinterpret_cast<uint4*>(buf + (int64_t)(z - z0) * kLo + c0 + mcb) = o;
  }
}

// the workgroup's walks for a wave group count G: walks in blocks of 2^lp aligned on the
// absolute walk index, each block in Gray order -- consecutive walks differ in one slice
// bit (6 + t), so a walk starts from the previous one's last state with planes 5 and 6 + t
// flipped: two XORs per group instead of the start state's twelve planes
template <int G>
__device__ __forceinline__ void seed_walks(const uint32_t (*pr)[kHiBits], const uint32_t* __restrict__ planes,
                                           uint32_t g0, int ng, int wng, uint8_t* st8, int tid, int co,
                                           const uint32_t* mx, int mcb, int c0, int z0, int z1,
                                           int8_t* __restrict__ buf, int lp) {
  const int wa = (z0 & ~(kWalk - 1)) >> kWalkBits, we = (z1 + kWalk - 1) >> kWalkBits, P = 1 << lp;
  const int b1 = (we + P - 1) >> lp;
  for (int b = (wa >> lp) + blockIdx.y; b < b1; b += gridDim.y) {
    uint32_t x[G];
    walk_start<G>(pr, (b << lp) << kWalkBits, x);
    for (int j = 0; j < P; ++j) {  // workgroup-uniform
      if (j) {
        const int t = __builtin_ctz(j);
#pragma unroll
        for (int g = 0; g < G; ++g) {
          uint32_t f = pr[g][kWalkBits - 1];
#pragma unroll
          for (int k = 0; k < kMaxWalkBlockBits; ++k)
            if (k == t) f ^= pr[g][kWalkBits + k];
          x[g] ^= f;
        }
      }
      const int w = (b << lp) + (j ^ (j >> 1));
      if (w < wa || w >= we) {  // outside the range: the state as if walked
#pragma unroll
        for (int g = 0; g < G; ++g) x[g] ^= pr[g][kWalkBits - 1];
        continue;
      }
      __syncthreads();  // the previous walk's store-out reads of `stage` are done
      walk_from<G>(pr, x, st8, co);
      seed_finish(planes, g0, ng, wng, st8, tid, co, mx, mcb, c0, w << kWalkBits, z0, z1, buf);
    }
  }
}

// 96 VGPRs: 5 waves per SIMD (the Gray-block state costs two more registers; at this bound the
// compiler spills one 8-byte value, reloaded once per walk)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5))) void seed_sm_kernel(
    const uint32_t* __restrict__ planes, const uint32_t* __restrict__ gofs, const uint32_t* __restrict__ off, int z0,
    int z1, int8_t* __restrict__ buf, int lp) {
  constexpr int NT = 256;
  __shared__ uint32_t stage[kWalk * NT / 4];
  uint8_t* st8 = reinterpret_cast<uint8_t*>(stage);
  const int tid = threadIdx.x;
  const int c0 = blockIdx.x * NT;
  // columns to lanes by group count (seed_lane_column); the stage rows and the store-out stay in
  // column order
  const int co = seed_lane_column(gofs, c0, tid);
  const int c = c0 + co;
  const uint32_t g0 = gofs[c];
  const int ng = (int)(gofs[c + 1] - g0);
  int wng = ng;
#pragma unroll
  for (int s = 32; s; s >>= 1) wng = max(wng, __shfl_xor(wng, s));
  uint32_t pr[kRegGroupsSM][kHiBits];
#pragma unroll
  for (int g = 0; g < kRegGroupsSM; ++g)
    if (g < ng) {
      load_planes(planes, (int64_t)g0 + g, pr[g]);
    } else {
#pragma unroll
      for (int k = 0; k < kHiBits; ++k) pr[g][k] = 0u;
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
  if (wng <= 1) seed_walks<1>(pr, planes, g0, ng, wng, st8, tid, co, mx, mcb, c0, z0, z1, buf, lp);
  else if (wng == 2) seed_walks<2>(pr, planes, g0, ng, wng, st8, tid, co, mx, mcb, c0, z0, z1, buf, lp);
  else seed_walks<3>(pr, planes, g0, ng, wng, st8, tid, co, mx, mcb, c0, z0, z1, buf, lp);
}

template <typename T>
__global__ __launch_bounds__(256) void seed_kernel(const uint32_t* __restrict__ planes,
                                                   const uint32_t* __restrict__ gofs,
                                                   const uint32_t* __restrict__ off, int z0, int z1,
                                                   T* __restrict__ buf) {
  seed_body<T>(planes, gofs, off, z0, z1, buf);
}

// LDS word of column e in the tile kernel: bits 2, 3, 4 XORed with bits 6, 5, 10, so the
// phase-1 b128 stores (8-lane groups: e bits 4..6 vary) and the phase-2 b32 loads (32-lane
// groups: e bits 0..3, 10 vary) are both conflict-free.
__device__ __forceinline__ int swz(int e) {
  return e ^ (((e >> 6) & 1) << 2) ^ (((e >> 5) & 1) << 3) ^ (((e >> 10) & 1) << 4);
}

// Butterfly over a lane bit without LDS: v_permlane{32,16}_swap brings the partner lane's
// value of register a into this lane's b (and b's into the partner), so the pair is
// combined in-lane.  Afterwards the lane bit and the register bit that told a from b have
// traded places.
__device__ __forceinline__ void lane_butterfly32(int32_t& a, int32_t& b) {
  const auto r = __builtin_amdgcn_permlane32_swap((unsigned)a, (unsigned)b, false, false);
  a = (int32_t)(r[0] + r[1]);
  b = (int32_t)(r[0] - r[1]);
}
__device__ __forceinline__ void lane_butterfly16(int32_t& a, int32_t& b) {
  const auto r = __builtin_amdgcn_permlane16_swap((unsigned)a, (unsigned)b, false, false);
  a = (int32_t)(r[0] + r[1]);
  b = (int32_t)(r[0] - r[1]);
}

// int16 / int32 seeds (columns of more than 127 codes: dense sets and multisets with heavy
// duplicates): per slice the WHT over the 14 column bits on the VALU, then S_w += F^2 by digit
// weight.  Persistent: workgroups stride over the chunk's slices.  Here sum_w S_w = 2^32 sum f^2
// can exceed 2^64, so every lane's per-slice sum (64 squares < 2^54 each: n <= 1e8) goes to the
// LDS bins as its two 32-bit halves (bins_lo / bins_hi never carry: < 2^26 adds each) and the
// bins to the counts' three limbs (add_weight_sum).
//   phase 1  registers q = e bits 0..3 + 16 * (12, 13); thread = e bits 4..11
//   phase 2  registers q = e bits 4..9;  lane = e bits 0..3, 10, 11; wave = e bits 12, 13
//   phase 3  lane bits 5, 4 (e 11, 10) by permlane swaps against q bits 1, 0 (e 5, 4):
//            then q = (e 10, 11, 6..9), lane = e bits 0..5, wave = e bits 12, 13 -- whole
//            2-bit digits, so an element's digit weight is thread constant + compile time.
template <typename T>
__global__ __launch_bounds__(256) void tile_kernel(const T* __restrict__ buf, int z0, int nslices,
                                                   unsigned long long* __restrict__ counts,
                                                   unsigned long long add_n,
                                                   const unsigned long long* __restrict__ sumsq) {
  static_assert(sizeof(T) >= 2, "int8 seeds take tile_reg_kernel");
  __shared__ int32_t lds[kLo];
  __shared__ unsigned long long bins_lo[17], bins_hi[17];
  constexpr int V = Chunk<T>::kVals, L = Chunk<T>::kLog;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid < 17) bins_lo[tid] = bins_hi[tid] = 0;
  const int t2 = (lane & 15) | ((lane >> 4) << 10) | (wave << 12);  // phase-2 e base
  const int wt_thread = digit_weight((uint32_t)lane | ((uint32_t)wave << 12));
  for (int s = blockIdx.x; s < nslices; s += gridDim.x) {
    const T* row = buf + (int64_t)s * kLo;
    int32_t x[64];
#pragma unroll
    for (int j = 0; j < Chunk<T>::kPerThread; ++j) {
      const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(row + tid * V + (j << (L + 8))));
      const T* e = reinterpret_cast<const T*>(&v);
#pragma unroll
      for (int r = 0; r < V; ++r) x[j * V + r] = e[r];
    }
    wht<64>(x);
    __syncthreads();  // the previous slice's phase-2 reads are done
#pragma unroll
    for (int q = 0; q < 64; q += 4)
      *reinterpret_cast<int4*>(lds + swz((q & 15) | (tid << 4) | ((q >> 4) << 12))) =
          make_int4(x[q], x[q + 1], x[q + 2], x[q + 3]);
    __syncthreads();
    const int a2 = swz(t2);
#pragma unroll
    for (int q = 0; q < 64; ++q) x[q] = lds[a2 ^ swz(q << 4)];
    wht<64>(x);
#pragma unroll
    for (int q = 0; q < 64; ++q)
      if (!(q & 2)) lane_butterfly32(x[q], x[q | 2]);  // e bit 11 <-> q bit 1 (e bit 5)
#pragma unroll
    for (int q = 0; q < 64; ++q)
      if (!(q & 1)) lane_butterfly16(x[q], x[q | 1]);  // e bit 10 <-> q bit 0 (e bit 4)
    unsigned long long acc[4] = {0, 0, 0, 0};
#pragma unroll
    for (int q = 0; q < 64; ++q)
      acc[digit_weight_c((uint32_t)(q & 3)) + digit_weight_c((uint32_t)(q >> 2))] +=
          (unsigned long long)((int64_t)x[q] * x[q]);
    const int w0 = digit_weight((uint32_t)(z0 + s)) + wt_thread;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (acc[k] & 0xFFFFFFFFull) atomicAdd(&bins_lo[w0 + k], acc[k] & 0xFFFFFFFFull);
      if (acc[k] >> 32) atomicAdd(&bins_hi[w0 + k], acc[k] >> 32);
    }
  }
  __syncthreads();
  if (tid < 17) add_weight_sum(counts, tid, bins_lo[tid], bins_hi[tid]);
  add_job_constants(counts, add_n, sumsq);
}

typedef int v4i_t __attribute__((ext_vector_type(4)));
typedef long v2l_t __attribute__((ext_vector_type(2)));
typedef short v2s_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ v2l_t pack_v2l(const uint32_t* w) {
  return v2l_t{(long)(((uint64_t)w[1] << 32) | w[0]), (long)(((uint64_t)w[3] << 32) | w[2])};
}

// ---------------------------------------------------------------- register-resident tile (int8 seeds)
// One WAVE transforms one whole slice with no LDS exchange and no barrier.  Column bits:
// P = 0..5 (digits 0-2), Q = 6..11 (digits 3-5), R = 12, 13 (digit 6).  Lane l's 16-B load
// (plane R, load mt) holds columns 16 (l >> 4) + 64 (l & 15) + 1024 mt + 4096 R + j: a wave
// reads each kilobyte of the slice whole.
//   stage 1 (per plane R): the bytes are the A operand of v_mfma_i32_16x16x64_i8 as loaded
//     (A[m = Q bits 0..3 = l & 15][k = P = 16 (l >> 4) + j]) against B = a quarter qn of H_64:
//     C1[m][n] = sum_P D * H -> transformed P' (n = P' bits 0..3 = l & 15, qn = bits 4, 5),
//     output rows m = 4 (l >> 4) + i.  So lane l holds Q bits 0, 1 = i, 2, 3 = l >> 4 and,
//     over the 4 loads, Q bits 4, 5 = mt: 16 values that ARE stage 2's B operand (k = 16 (l >> 4)
//     + 4 mt + i, a relabeling of whole Q digits), packed into bytes in registers.
//   stage 2: H_64 over Q (A = the same H quarters).  |v + 128| < 2^15 needs two bytes: with
//     y = v + 128 = 256 h + l', v = 256 h + (l' - 128), so H v = (H h << 8) + H (l' - 128): two
//     i8 MFMAs per output tile, the first shifted into the second's accumulator.  The byte
//     split goes through int16 pairs (one v_perm packs two stage-1 outputs), which are also
//     what the plane sums accumulate (v_pk_add_u16; the sum over the planes of v + 128 from
//     -384 stays within +-32,640).  Outputs Q' rows 16 q2 + 4 (l >> 4) + i2: whole digits.
//   R (one base digit) by Parseval instead of a butterfly: with G_R = the 12-bit transform of
//     plane R and F(R') = sum_R (-1)^<R, R'> G_R,  F(0) = transform of sum_R D_R = sum_R C1_R
//     (added after stage 1) and sum_{R' != 0} F(R')^2 = 4 sum_R G_R^2 - F(0)^2.  So every
//     (P', Q') adds F(0)^2 to weight w and 4 sum G_R^2 - F(0)^2 to weight w + 1: five stage-2
//     transforms per slice (4 planes + the sum), no exchange between planes.
//   Two quarters' MFMA chains are interleaved per wave (stage 1 of both, both byte splits, both
//     high-byte and both low-byte stage-2 groups, then both sets of squares), and the next
//     plane's loads are in flight while this one is transformed: 167 VGPRs, 3 waves per SIMD.
// Weight of (P', Q', R'): digits of l & 3, (l >> 2) & 3, l >> 4 (thread constant) + qn + q2
// + i2 (compile time) + the slice's + [R' != 0].  Each wave of the grid takes a contiguous run
// of slice positions; position u is slice order[u] (a whole aligned chunk sorted by digit
// weight, so the run's weight changes rarely and F^2 is binned in registers) or u.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void tile_reg_kernel(
    const int8_t* __restrict__ buf, const uint16_t* __restrict__ order, int z0, int nslices,
    unsigned long long* __restrict__ counts, unsigned long long add_n, const unsigned long long* __restrict__ sumsq) {
  // int8 seeds: every column holds <= 127 codes, so sum_w S_w = 2^32 sum f^2 <= 2^32 * 2^14 * 127^2
  // < 2^62 and 64-bit register / LDS sums cannot wrap
  __shared__ unsigned long long bins[17];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid < 17) bins[tid] = 0;
  __syncthreads();
  v2l_t H[4];  // H_64 rows 16 q + (l & 15), columns 16 (l >> 4) + j: stage 1's B and stage 2's A
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
    H[q] = v2l_t{(long)(((uint64_t)w[1] << 32) | w[0]), (long)(((uint64_t)w[3] << 32) | w[2])};
  }
  const int wt_thread = digit_weight((uint32_t)(lane & 15)) + digit_weight((uint32_t)(lane >> 4));
  const int lane_off = 16 * (lane >> 4) + 64 * (lane & 15);
  const int gw = blockIdx.x * 4 + wave, GW = gridDim.x * 4;
  const int ub = (int)((int64_t)nslices * gw / GW), ue = (int)((int64_t)nslices * (gw + 1) / GW);
  // the squares of the two interleaved quarters go to separate sums (two dependency chains per
  // weight instead of one), added at the flush
  unsigned long long accA[4] = {0, 0, 0, 0}, accB[4] = {0, 0, 0, 0}, accB2[4] = {0, 0, 0, 0};
  int cur_w = -1;
  auto flush = [&]() {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (accA[k]) atomicAdd(&bins[cur_w + wt_thread + k], accA[k]);
      const unsigned long long b = 4 * (accB[k] + accB2[k]) - accA[k];
      if (b) atomicAdd(&bins[cur_w + wt_thread + k + 1], b);
      accA[k] = 0;
      accB[k] = 0;
      accB2[k] = 0;
    }
  };
  auto load_plane = [&](int sl, int R, v2l_t* dst) {
    const int8_t* p = buf + (int64_t)sl * kLo + lane_off + 4096 * R;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
      dst[mt] = __builtin_nontemporal_load(reinterpret_cast<const v2l_t*>(p + 1024 * mt));
  };
  // two quarters qa, qb of stage 2 from their byte splits, then their squares
  auto stage2x2B = [&](const v2l_t& Bla, const v2l_t& Bha, const v2l_t& Blb, const v2l_t& Bhb, auto qa_c,
                       auto qb_c, unsigned long long* acc, unsigned long long* acc2) {
    constexpr int qa = decltype(qa_c)::value, qb = decltype(qb_c)::value;
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
#ifdef SCT_TILE_SQ_ABL
        // timing-only ablation (wrong results): the squares replaced by one full-rate XOR, the floor
        // of any exact F^2 accumulate (ab_tile_squares_r06)
        acc[digit_weight_c((uint32_t)qa) + digit_weight_c((uint32_t)q2) + digit_weight_c((uint32_t)i)] ^=
            (uint32_t)ca[q2][i];
        acc2[digit_weight_c((uint32_t)qb) + digit_weight_c((uint32_t)q2) + digit_weight_c((uint32_t)i)] ^=
            (uint32_t)cb[q2][i];
#else
        acc[digit_weight_c((uint32_t)qa) + digit_weight_c((uint32_t)q2) + digit_weight_c((uint32_t)i)] +=
            (unsigned long long)((int64_t)ca[q2][i] * ca[q2][i]);
        acc2[digit_weight_c((uint32_t)qb) + digit_weight_c((uint32_t)q2) + digit_weight_c((uint32_t)i)] +=
            (unsigned long long)((int64_t)cb[q2][i] * cb[q2][i]);
#endif
      }
  };
  // int16 pairs (v + 128 of stage 1, |.| < 2^15) -> the high / low byte operands
  auto split16 = [&](const uint32_t (*pr)[2], v2l_t& Bl, v2l_t& Bh) {
    uint32_t lo[4], hi[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      lo[mt] = __builtin_amdgcn_perm(pr[mt][1], pr[mt][0], 0x06040200u) ^ 0x80808080u;
      hi[mt] = __builtin_amdgcn_perm(pr[mt][1], pr[mt][0], 0x07050301u);
    }
    Bl = pack_v2l(lo);
    Bh = pack_v2l(hi);
  };
  auto pairs16 = [&](const v4i_t* c1, uint32_t (*pr)[2]) {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      pr[mt][0] = __builtin_amdgcn_perm((uint32_t)c1[mt][1], (uint32_t)c1[mt][0], 0x05040100u);
      pr[mt][1] = __builtin_amdgcn_perm((uint32_t)c1[mt][3], (uint32_t)c1[mt][2], 0x05040100u);
    }
  };
  // planes in turn (a runtime loop: one plane's 16 VGPRs of bytes live at a time, the next
  // plane's loads in flight), the per-plane sums of all four quarters carried across
  for (int u = ub; u < ue; ++u) {
    // (a chunk of 2^k > kMaxOrder slices: each aligned 2^16 block in its own weight order)
    const int s = order ? ((u & ~(kMaxOrder - 1)) | (int)order[u & (kMaxOrder - 1)]) : u;
    const int wz = digit_weight((uint32_t)(z0 + s));  // wave-uniform
    if (wz != cur_w) {
      if (cur_w >= 0) flush();
      cur_w = wz;
    }
    uint32_t csp[4][4][2];  // [qn][mt]: sum over the planes of v + 128 as int16 pairs, from -384
#pragma unroll
    for (int qn = 0; qn < 4; ++qn)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) csp[qn][mt][0] = csp[qn][mt][1] = 0xFE80FE80u;
    v2l_t dn[4];
    load_plane(s, 0, dn);
#pragma unroll 1
    for (int R = 0; R < 4; ++R) {
      v2l_t d[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) d[mt] = dn[mt];
      if (R < 3) load_plane(s, R + 1, dn);
      auto quarters16 = [&](auto qa_c, auto qb_c) {
        constexpr int qa = decltype(qa_c)::value, qb = decltype(qb_c)::value;
        v4i_t c1a[4], c1b[4];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          c1a[mt] = __builtin_amdgcn_mfma_i32_16x16x64_i8(d[mt], H[qa], v4i_t{128, 128, 128, 128}, 0, 0, 0);
          c1b[mt] = __builtin_amdgcn_mfma_i32_16x16x64_i8(d[mt], H[qb], v4i_t{128, 128, 128, 128}, 0, 0, 0);
        }
        uint32_t pa[4][2], pb[4][2];
        pairs16(c1a, pa);
        pairs16(c1b, pb);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            csp[qa][mt][h] = __builtin_bit_cast(uint32_t, __builtin_bit_cast(v2s_t, csp[qa][mt][h]) +
                                                              __builtin_bit_cast(v2s_t, pa[mt][h]));
            csp[qb][mt][h] = __builtin_bit_cast(uint32_t, __builtin_bit_cast(v2s_t, csp[qb][mt][h]) +
                                                              __builtin_bit_cast(v2s_t, pb[mt][h]));
          }
        v2l_t Bla, Bha, Blb, Bhb;
        split16(pa, Bla, Bha);
        split16(pb, Blb, Bhb);
        stage2x2B(Bla, Bha, Blb, Bhb, qa_c, qb_c, accB, accB2);
        __builtin_amdgcn_sched_barrier(0);
      };
      quarters16(std::integral_constant<int, 0>(), std::integral_constant<int, 1>());
      quarters16(std::integral_constant<int, 2>(), std::integral_constant<int, 3>());
    }
    v2l_t Bla, Bha, Blb, Bhb;
    split16(csp[0], Bla, Bha);
    split16(csp[1], Blb, Bhb);
    stage2x2B(Bla, Bha, Blb, Bhb, std::integral_constant<int, 0>(), std::integral_constant<int, 1>(), accA, accA);
    split16(csp[2], Bla, Bha);
    split16(csp[3], Blb, Bhb);
    stage2x2B(Bla, Bha, Blb, Bhb, std::integral_constant<int, 2>(), std::integral_constant<int, 3>(), accA, accA);
  }
  if (cur_w >= 0) flush();
  __syncthreads();
  if (tid < 17) add_weight_sum64(counts, tid, bins[tid]);
  add_job_constants(counts, add_n, sumsq);
}

// sum f^2 (ensure_sumsq): SPECTRAL codes are < 2^32, so the low 32 bits are the code
__global__ void low32_kernel(const uint64_t* __restrict__ codes, int64_t n, uint32_t* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (uint32_t)codes[i];
}

// sorted codes: sum over i of 2 r_i + 1, r_i = #{j < i : key j = key i} (a code of multiplicity f
// adds 1 + 3 + ... + 2f - 1 = f^2); r_i by a lower-bound search when the left neighbour is equal
__global__ __launch_bounds__(256) void sumsq_kernel(const uint32_t* __restrict__ sorted, int64_t n,
                                                    unsigned long long* __restrict__ out) {
  unsigned long long acc = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t v = sorted[i];
    int64_t r = 0;
    if (i > 0 && sorted[i - 1] == v) {
      int64_t a = 0, b = i - 1;  // first index holding v lies in [a, b]
      while (a < b) {
        const int64_t m = (a + b) >> 1;
        if (sorted[m] < v) a = m + 1;
        else b = m;
      }
      r = i - a;
    }
    acc += 2 * (unsigned long long)r + 1;
  }
#pragma unroll
  for (int s = 32; s; s >>= 1) acc += __shfl_xor(acc, s);
  if ((threadIdx.x & 63) == 0 && acc) atomicAdd(out, acc);
}

// the plan's probe (one pass over the codes): their OR, and the code counts of every 14- and
// 16-bit column (global atomics: 737K codes over 2^14 / 2^16 counters barely contend)
__global__ __launch_bounds__(256) void probe_kernel(const uint64_t* __restrict__ codes, int64_t n,
                                                    uint32_t* __restrict__ cnt14, uint32_t* __restrict__ cnt16,
                                                    unsigned long long* __restrict__ out) {
  unsigned long long o = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t x = codes[i];
    o |= x;
    atomicAdd(&cnt14[x & (kLo - 1)], 1u);
    atomicAdd(&cnt16[x & 0xFFFFu], 1u);
  }
#pragma unroll
  for (int s = 32; s; s >>= 1) o |= __shfl_xor(o, s);
  if ((threadIdx.x & 63) == 0 && o) atomicOr(out, o);
}
// The 14-bit column counts without global atomics (sets of >= kProbeHistMin codes): workgroup g
// counts its contiguous share in LDS (as column_hist_wg_kernel) and writes H[g][.], ORing the
// codes on the way; probe_max14_kernel sums each column over the workgroups and takes the max.
// The 16-bit counts (only asked for when 14-bit columns would need int16 seeds, or forced) keep
// the atomic probe_kernel below.
constexpr int64_t kProbeHistMin = 1 << 17;
__global__ __launch_bounds__(kSortThreads) void probe_hist14_kernel(const uint64_t* __restrict__ codes, int64_t n,
                                                                    uint32_t* __restrict__ H,
                                                                    unsigned long long* __restrict__ out) {
  __shared__ uint32_t h[kLo];
  for (int c = threadIdx.x; c < kLo; c += kSortThreads) h[c] = 0;
  __syncthreads();
  int64_t b, e;
  wg_range(n, b, e);
  unsigned long long o = 0;
  for (int64_t i = b + threadIdx.x; i < e; i += kSortThreads) {
    const uint64_t x = codes[i];
    o |= x;
    atomicAdd(&h[x & (kLo - 1)], 1u);
  }
#pragma unroll
  for (int s = 32; s; s >>= 1) o |= __shfl_xor(o, s);
  if ((threadIdx.x & 63) == 0 && o) atomicOr(out, o);
  __syncthreads();
  uint32_t* row = H + (int64_t)blockIdx.x * kLo;
  for (int c = threadIdx.x; c < kLo; c += kSortThreads) row[c] = h[c];
}

__global__ __launch_bounds__(256) void probe_max14_kernel(const uint32_t* __restrict__ H, int wgs,
                                                          unsigned long long* __restrict__ out) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  uint32_t m = 0;
#pragma unroll 8
  for (int g = 0; g < wgs; ++g) m += H[(int64_t)g * kLo + c];
#pragma unroll
  for (int s = 32; s; s >>= 1) m = max(m, (uint32_t)__shfl_xor(m, s));
  if ((threadIdx.x & 63) == 0 && m) atomicMax(out + 1, (unsigned long long)m);
}

// out[1] = max cnt14, out[2] = max cnt16 (grid covers the 2^16 counters)
__global__ __launch_bounds__(256) void probe_max_kernel(const uint32_t* __restrict__ cnt14,
                                                        const uint32_t* __restrict__ cnt16,
                                                        unsigned long long* __restrict__ out) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  unsigned m14 = c < kLo ? cnt14[c] : 0u, m16 = cnt16[c];
#pragma unroll
  for (int s = 32; s; s >>= 1) {
    m14 = max(m14, (unsigned)__shfl_xor(m14, s));
    m16 = max(m16, (unsigned)__shfl_xor(m16, s));
  }
  if ((threadIdx.x & 63) == 0) {
    if (m14) atomicMax(out + 1, (unsigned long long)m14);
    if (m16) atomicMax(out + 2, (unsigned long long)m16);
  }
}

template <typename T>
int launch_seed(State& st, int z0, int z1, hipStream_t s) {
  T* buf = reinterpret_cast<T*>(st.d_buf);
  const int walks = (z1 - (z0 & ~(kWalk - 1)) + kWalk - 1) / kWalk;
  // 16 walks per workgroup for a full chunk (measured best at 65,536 slices); smaller chunks
  // keep >= 64 workgroup rows so the grid still fills the chip
  const int per_wg = std::max(1, std::min(kSeedWalks, walks / 64));
  const dim3 sgrid(kLo / 256, (unsigned)((walks + per_wg - 1) / per_wg));
  if constexpr (sizeof(T) == 1) {
    int lp = 0;  // walks per Gray-ordered block: the largest power of two <= per_wg, <= 16
    while (lp < kMaxWalkBlockBits && (2 << lp) <= per_wg) ++lp;
    const int wa = (z0 & ~(kWalk - 1)) / kWalk, we = (z1 + kWalk - 1) / kWalk;
    const int nb = ((we + (1 << lp) - 1) >> lp) - (wa >> lp);
    hipLaunchKernelGGL(seed_sm_kernel, dim3(kLo / 256, (unsigned)nb), dim3(256), 0, s, st.d_planes, st.d_gofs, st.d_off,
                       z0, z1, buf, lp);
  } else
    hipLaunchKernelGGL(seed_kernel<T>, sgrid, dim3(256), 0, s, st.d_planes, st.d_gofs, st.d_off, z0, z1, buf);
  SCT_LAUNCH_CHECK();
  return SCT_OK;
}

template <typename T>
int launch_tile(State& st, int z0, int z1, unsigned long long* counts, hipStream_t s, unsigned long long add_n = 0) {
  T* buf = reinterpret_cast<T*>(st.d_buf);
  if constexpr (sizeof(T) == 1) {
    // an aligned power-of-two range goes in digit-weight order (table 2^b at offset 2^b)
    const int ns = z1 - z0;
    const uint16_t* order = ((ns & (ns - 1)) == 0 && z0 % ns == 0) ? st.d_order + std::min(ns, kMaxOrder) : nullptr;
    const dim3 rgrid((unsigned)std::max(1, std::min(st.grid * st.tile_wgs, (z1 - z0 + 3) / 4)));
    hipLaunchKernelGGL(tile_reg_kernel, rgrid, dim3(256), 0, s, buf, order, z0, z1 - z0, counts, add_n,
                       st.sumsq_ptr());
  } else {
    const dim3 grid((unsigned)std::min(st.grid * 2, z1 - z0));
    hipLaunchKernelGGL(tile_kernel<T>, grid, dim3(256), 0, s, buf, z0, z1 - z0, counts, add_n,
                       st.sumsq_ptr());
  }
  SCT_LAUNCH_CHECK();
  return SCT_OK;
}

template <typename T>
int launch_chunk(State& st, int z0, int z1, unsigned long long* counts, hipStream_t s, unsigned long long add_n) {
  hipEvent_t t0 = st.timer ? st.timer->start(s) : nullptr;
  int rc = launch_seed<T>(st, z0, z1, s);
  if (st.timer) st.timer->stop(s, t0, sct::LaunchTimer::SEED);
  if (rc != SCT_OK) return rc;
  t0 = st.timer ? st.timer->start(s) : nullptr;
  rc = launch_tile<T>(st, z0, z1, counts, s, add_n);
  if (st.timer) st.timer->stop(s, t0, sct::LaunchTimer::TILE);
  return rc;
}

// Bench aid: seed and tile kernels timed apart, each as `repeats` back-to-back launches on
// one chunk bracketed by HIP events (the timestamps of events between dependent kernels of
// one stream do not split the kernels reliably).  counts receives garbage.
template <typename T>
int time_chunk(State& st, int z0, int z1, unsigned long long* counts, int repeats, hipStream_t s,
               double* seed_ms, double* tile_ms) {
  hipEvent_t e[3];
  for (auto& x : e) SCT_HIP(hipEventCreate(&x));
  struct Free {
    hipEvent_t* e;
    ~Free() {
      for (int i = 0; i < 3; ++i) (void)hipEventDestroy(e[i]);
    }
  } guard{e};
  int rc = launch_seed<T>(st, z0, z1, s);  // warm
  if (rc == SCT_OK) rc = launch_tile<T>(st, z0, z1, counts, s);
  SCT_HIP(hipEventRecord(e[0], s));
  for (int r = 0; rc == SCT_OK && r < repeats; ++r) rc = launch_seed<T>(st, z0, z1, s);
  SCT_HIP(hipEventRecord(e[1], s));
  for (int r = 0; rc == SCT_OK && r < repeats; ++r) rc = launch_tile<T>(st, z0, z1, counts, s);
  SCT_HIP(hipEventRecord(e[2], s));
  if (rc != SCT_OK) return rc;
  SCT_HIP(hipEventSynchronize(e[2]));
  float a = 0, b = 0;
  SCT_HIP(hipEventElapsedTime(&a, e[0], e[1]));
  SCT_HIP(hipEventElapsedTime(&b, e[1], e[2]));
  *seed_ms = a / repeats;
  *tile_ms = b / repeats;
  return SCT_OK;
}

}  // namespace

// ---------------------------------------------------------------- plan cache (workspace)
struct Workspace {
  int device = -1;
  bool busy = false;
  bool release = false;  // sct_allpairs_cache_release() while lent out: free on return
  bool order_ready = false;
  void* p[W_NSLOTS] = {};
  size_t cap[W_NSLOTS] = {};
  // a plan's private arena (SCT_ALLPAIRS_NO_CACHE): one block, the slots carved from it in turn,
  // freed whole when the plan goes -- one hipMalloc / hipFree per call instead of one per slot
  // (a hipFree costs ~110 us, profiles/dropin_hip_api_r06.csv); slots that do not fit get their own
  bool arena = false;
  uint8_t* base = nullptr;
  size_t size = 0, used = 0;
  std::vector<void*> extra;
};

namespace {
std::mutex g_ws_mu;
Workspace* g_ws[64] = {};

void ws_free(Workspace* ws) {
  if (ws->arena) {
    if (ws->base) (void)hipFree(ws->base);
    for (void* q : ws->extra) (void)hipFree(q);
  } else {
    for (int k = 0; k < W_NSLOTS; ++k)
      if (ws->p[k]) (void)hipFree(ws->p[k]);
  }
  delete ws;
}
}  // namespace

Workspace* ws_arena(size_t bytes) {
  auto* ws = new Workspace();
  ws->arena = true;
  ws->busy = true;
  if (hipGetDevice(&ws->device) != hipSuccess || hipMalloc((void**)&ws->base, bytes) != hipSuccess) {
    (void)hipGetLastError();  // (no block: every slot its own allocation, as without an arena)
    ws->base = nullptr;
    bytes = 0;
  }
  ws->size = bytes;
  return ws;
}

Workspace* ws_acquire() {
  if (sct::tune(SCT_TUNE_PLAN_CACHE, 1) == 0) return nullptr;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> lk(g_ws_mu);
  Workspace*& ws = g_ws[dev];
  if (!ws) {
    ws = new Workspace();
    ws->device = dev;
  }
  if (ws->busy) return nullptr;
  ws->busy = true;
  ws->release = false;
  return ws;
}

void ws_release(Workspace* ws) {
  if (!ws) return;
  if (ws->arena) {
    ws_free(ws);
    return;
  }
  std::lock_guard<std::mutex> lk(g_ws_mu);
  ws->busy = false;
  if (ws->release) {
    g_ws[ws->device] = nullptr;
    ws_free(ws);
  }
}

int ws_get(Workspace* ws, int slot, size_t bytes, void** p) {
  bytes = std::max<size_t>(bytes, 256);
  if (!ws) {
    SCT_HIP(hipMalloc(p, bytes));
    return SCT_OK;
  }
  if (ws->arena) {
    if (ws->cap[slot] < bytes) {
      const size_t at = (ws->used + 255) & ~(size_t)255;
      if (ws->base && at + bytes <= ws->size) {
        ws->p[slot] = ws->base + at;
        ws->used = at + bytes;
      } else {
        void* q = nullptr;
        SCT_HIP(hipMalloc(&q, bytes));
        ws->extra.push_back(q);
        ws->p[slot] = q;
      }
      ws->cap[slot] = bytes;
      if (slot == W_ORDER) ws->order_ready = false;
    }
    *p = ws->p[slot];
    return SCT_OK;
  }
  if (ws->cap[slot] < bytes) {  // grow (rare: a larger set than any before on this device)
    if (ws->p[slot]) (void)hipFree(ws->p[slot]);
    ws->p[slot] = nullptr;
    ws->cap[slot] = 0;
    if (slot == W_ORDER) ws->order_ready = false;
    SCT_HIP(hipMalloc(&ws->p[slot], bytes));
    ws->cap[slot] = bytes;
  }
  *p = ws->p[slot];
  return SCT_OK;
}

void ws_put(Workspace* ws, void* p) {
  if (!ws && p) (void)hipFree(p);
}

bool* ws_order_ready(Workspace* ws) { return ws ? &ws->order_ready : nullptr; }

void ws_release_all() {
  std::lock_guard<std::mutex> lk(g_ws_mu);
  for (auto& ws : g_ws) {
    if (!ws) continue;
    if (ws->busy) {
      ws->release = true;
      continue;
    }
    int cur = 0;
    const bool dev_ok = hipGetDevice(&cur) == hipSuccess && hipSetDevice(ws->device) == hipSuccess;
    ws_free(ws);
    if (dev_ok) (void)hipSetDevice(cur);
    ws = nullptr;
  }
}

void note_stream(State& st, hipStream_t s) {
  for (auto& u : st.used)
    if (u.first == s) {
      (void)hipEventRecord(u.second, s);
      return;
    }
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return;
  (void)hipEventRecord(e, s);
  st.used.emplace_back(s, e);
}

int make_order_table(State& st) {
  // for every power of two L <= 2^16: the offsets [0, L) sorted by digit weight, stored
  // at [L, 2L) (an aligned range of L slices adds a constant weight to all of them); the
  // same for every plan, so sorted once per process and uploaded once per workspace
  static const std::vector<uint16_t> order = [] {
    std::vector<uint16_t> o(2 * kMaxOrder);
    for (int len = 1; len <= kMaxOrder; len *= 2) {  // a stable counting sort by weight (0..8)
      int start[10] = {};
      for (int u = 0; u < len; ++u) ++start[digit_weight_c((uint32_t)u) + 1];
      for (int w = 1; w < 10; ++w) start[w] += start[w - 1];
      uint16_t* b = o.data() + len;
      for (int u = 0; u < len; ++u) b[start[digit_weight_c((uint32_t)u)]++] = (uint16_t)u;
    }
    return o;
  }();
  void* p = nullptr;
  if (int rc = ws_get(st.ws, W_ORDER, order.size() * 2, &p); rc != SCT_OK) return rc;
  st.d_order = reinterpret_cast<uint16_t*>(p);
  bool* ready = ws_order_ready(st.ws);
  if (!ready || !*ready) {
    SCT_HIP(hipMemcpy(st.d_order, order.data(), order.size() * 2, hipMemcpyHostToDevice));
    if (ready) *ready = true;
  }
  return SCT_OK;
}

int probe(Workspace* ws, const uint64_t* d_codes, int64_t n, unsigned long long* out) {
  void* p = nullptr;
  constexpr size_t kWords = (size_t)kLo + (1u << 16);
  const bool hist = n >= kProbeHistMin;  // (smaller sets: the atomic counts are as quick)
  const size_t hbytes = hist ? (size_t)kSortWGs * kLo * 4 : 0;
  if (int rc = ws_get(ws, W_PROBE, hbytes + kWords * 4 + 32, &p); rc != SCT_OK) return rc;
  struct Put {
    Workspace* ws;
    void* p;
    ~Put() { ws_put(ws, p); }
  } put{ws, p};
  uint32_t* H = reinterpret_cast<uint32_t*>(p);
  uint32_t* cnt14 = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(p) + hbytes);
  uint32_t* cnt16 = cnt14 + kLo;
  unsigned long long* res = reinterpret_cast<unsigned long long*>(cnt16 + (1u << 16));
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(1024, sct::ceil_div(n, 256)));
  if (hist) {
    // OR and the 14-bit counts first; the 16-bit ones only when the 14-bit layout cannot take
    // int8 seeds (or 16-bit columns are forced: SCT_TUNE_SPECTRAL_COLUMNS)
    SCT_HIP(hipMemsetAsync(res, 0, 32, 0));
    hipLaunchKernelGGL(probe_hist14_kernel, dim3(kSortWGs), dim3(kSortThreads), 0, 0, d_codes, n, H, res);
    SCT_LAUNCH_CHECK();
    hipLaunchKernelGGL(probe_max14_kernel, dim3(kLo / 256), dim3(256), 0, 0, H, kSortWGs, res);
    SCT_LAUNCH_CHECK();
    SCT_HIP(hipMemcpy(out, res, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    if (out[1] <= 127 && sct::tune(SCT_TUNE_SPECTRAL_COLUMNS, 0) != kLoBits16) return SCT_OK;  // (out[2] = 0: unused)
  }
  SCT_HIP(hipMemsetAsync(cnt14, 0, kWords * 4 + 32, 0));
  if (n > 0) {
    hipLaunchKernelGGL(probe_kernel, dim3(blocks), dim3(256), 0, 0, d_codes, n, cnt14, cnt16, res);
    SCT_LAUNCH_CHECK();
    hipLaunchKernelGGL(probe_max_kernel, dim3((1u << 16) / 256), dim3(256), 0, 0, cnt14, cnt16, res);
    SCT_LAUNCH_CHECK();
  }
  SCT_HIP(hipMemcpy(out, res, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  return SCT_OK;
}

int alloc_buf(State& st, int64_t* chunk, int64_t min_chunk, size_t bytes_per_slice) {
  for (;;) {
    const size_t bytes = (size_t)((*chunk + 15) & ~15ll) * bytes_per_slice;  // whole 16-slice groups
    const int rc = ws_get(st.ws, W_BUF, bytes, &st.d_buf);
    if (rc == SCT_OK) {
      st.buf_bytes = bytes;
      return SCT_OK;
    }
    (void)hipGetLastError();  // clear the out-of-memory state
    if (rc != SCT_E_NOMEM || *chunk / 2 < min_chunk) return rc;
    *chunk /= 2;
  }
}

int create(State& st, const uint64_t* d_codes, int64_t n, int64_t chunk, int cus, unsigned max14, unsigned max16) {
  st.n = n;
  st.chunk = std::max<int64_t>(kWalk, std::min<int64_t>(chunk, kSlices));
  st.grid = std::max(1, cus);  // CUs; the tile kernels' persistent grids are sized from it
  if (n < 2) return SCT_OK;
  // the densest column bounds |seed| and so the intermediate's width (the codes are fixed
  // for the plan's life); a set too dense for int8 seeds on 14-bit columns takes 16-bit
  // columns when every one of those holds <= 127 codes (spectral16.hip)
  const unsigned maxm = max14;
  const int64_t force = sct::tune(SCT_TUNE_SPECTRAL_COLUMNS, 0);
  if (((maxm > 127 && force != kLoBits) || force == kLoBits16) && max16 <= 127)
    return create16(st, d_codes, n, max16, chunk, cus);
  void* p = nullptr;
  auto get = [&](int slot, size_t bytes, auto** out) {
    const int rc = ws_get(st.ws, slot, bytes, &p);
    if (rc == SCT_OK) *out = reinterpret_cast<std::remove_reference_t<decltype(**out)>*>(p);
    return rc;
  };
  if (int rc = get(W_HI, (size_t)n * 4, &st.d_hi); rc != SCT_OK) return rc;
  if (int rc = get(W_OFF, (size_t)(kLo + 1) * 4, &st.d_off); rc != SCT_OK) return rc;
  if (int rc = get(W_CNT, (size_t)2 * kLo * 4, &st.d_cnt); rc != SCT_OK) return rc;  // counts, then cursors
  st.max_m = maxm;
  st.elem_bytes = maxm <= 127 ? 1 : (maxm <= 32767 ? 2 : 4);
  // the intermediate holds one chunk: at most 4 GiB (all 2^18 slices at int8: one seed and one
  // tile launch per count; int16 / int32 seeds take 2 / 4 passes)
  st.chunk = std::min<int64_t>(st.chunk, (int64_t(4) << 30) / ((int64_t)kLo * st.elem_bytes));
  static const int per_cu = [] {  // resident register-tile workgroups per CU (VGPR bound: 3)
    int v = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, tile_reg_kernel, 256, 0) != hipSuccess || v <= 0) v = 2;
    return v;
  }();
  st.tile_wgs = per_cu;
  if (int rc = make_order_table(st); rc != SCT_OK) return rc;
  st.max_groups = sct::ceil_div(n, 32) + kLo;
  if (int rc = get(W_GOFS, (size_t)(kLo + 1) * 4, &st.d_gofs); rc != SCT_OK) return rc;
  if (int rc = get(W_HIST, (size_t)kSortWGs * kLo * 4, &st.d_hist); rc != SCT_OK) return rc;
  if (int rc = get(W_PLANES, (size_t)st.max_groups * kPlaneWords * 4, &st.d_planes); rc != SCT_OK) return rc;
  if (int rc = alloc_buf(st, &st.chunk, std::min<int64_t>(st.chunk, 4096), (size_t)kLo * st.elem_bytes); rc != SCT_OK)
    return rc;
  if (int rc = get(W_SUMSQ, sizeof(unsigned long long), &st.d_sumsq); rc != SCT_OK) return rc;
  return SCT_OK;
}

void wait_idle(State& st) {
  for (auto& u : st.used) {
    (void)hipEventSynchronize(u.second);
    (void)hipEventDestroy(u.second);
  }
  st.used.clear();
}

void destroy(State& st) {
  // the plan's work has to be done before its buffers serve another plan (or are freed)
  wait_idle(st);
  for (void* p : {(void*)st.d_hi, (void*)st.d_off, (void*)st.d_cnt, (void*)st.d_gofs, (void*)st.d_planes,
                  (void*)st.d_hist, st.d_buf, (void*)st.d_order, (void*)st.d_sumsq, st.d_sumsq_tmp})
    ws_put(st.ws, p);
  ws_release(st.ws);
  st = State();
}

int ensure_sumsq(State& st, const uint64_t* d_codes, hipStream_t s) {
  if (st.sumsq_ready || st.distinct) return SCT_OK;
  // scratch: low 32 bits (4n), sorted (4n), radix-sort temp
  size_t tmp = 0;
  SCT_HIP(hipcub::DeviceRadixSort::SortKeys(nullptr, tmp, (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)st.n, 0,
                                            32, s));
  const size_t keys = ((size_t)st.n * 4 + 255) & ~(size_t)255;
  const size_t need = 2 * keys + tmp;
  char* base = reinterpret_cast<char*>(st.d_buf);
  if (need > st.buf_bytes) {  // a small test chunk: scratch of its own, kept for the plan's life
    if (int rc = ws_get(st.ws, W_SUMSQ_TMP, need, &st.d_sumsq_tmp); rc != SCT_OK) return rc;
    base = reinterpret_cast<char*>(st.d_sumsq_tmp);
  }
  uint32_t* k0 = reinterpret_cast<uint32_t*>(base);
  uint32_t* k1 = reinterpret_cast<uint32_t*>(base + keys);
  const int blocks = (int)std::min<int64_t>(2048, sct::ceil_div(st.n, 256));
  hipLaunchKernelGGL(low32_kernel, dim3(blocks), dim3(256), 0, s, d_codes, st.n, k0);
  SCT_LAUNCH_CHECK();
  SCT_HIP(hipcub::DeviceRadixSort::SortKeys(base + 2 * keys, tmp, k0, k1, (int)st.n, 0, 32, s));
  SCT_HIP(hipMemsetAsync(st.d_sumsq, 0, sizeof(unsigned long long), s));
  hipLaunchKernelGGL(sumsq_kernel, dim3(blocks), dim3(256), 0, s, k1, st.n, st.d_sumsq);
  SCT_LAUNCH_CHECK();
  st.sumsq_ready = true;
  return SCT_OK;
}

int build(State& st, const uint64_t* d_codes, hipStream_t s) {
  if (st.n < 2) return SCT_OK;
  if (int rc = ensure_sumsq(st, d_codes, s); rc != SCT_OK) return rc;
  if (st.lo_bits == kLoBits16) return build16(st, d_codes, s);
  hipEvent_t t0 = st.timer ? st.timer->start(s) : nullptr;
  hipLaunchKernelGGL(column_hist_wg_kernel, dim3(kSortWGs), dim3(kSortThreads), 0, s, d_codes, st.n, st.d_hist);
  SCT_LAUNCH_CHECK();
  hipLaunchKernelGGL(column_prefix_kernel, dim3(kLo / 256), dim3(256), 0, s, st.d_hist, kSortWGs, st.d_cnt);
  SCT_LAUNCH_CHECK();
  hipLaunchKernelGGL(column_scan16_kernel, dim3(1), dim3(1024), 0, s, st.d_cnt, st.d_off, st.d_gofs);
  SCT_LAUNCH_CHECK();
  hipLaunchKernelGGL(column_scatter_wg_kernel, dim3(kSortWGs), dim3(kSortThreads), 0, s, d_codes, st.n, st.d_hist,
                     st.d_off, st.d_hi);
  SCT_LAUNCH_CHECK();
  if (st.max_m <= 128) {
    hipLaunchKernelGGL(planes_slot_kernel<4>, dim3(kLo * 4 / 256), dim3(256), 0, s, st.d_hi, st.d_off, st.d_gofs,
                       st.max_groups, st.d_planes);
  } else {
    hipLaunchKernelGGL(planes_kernel, dim3((unsigned)sct::ceil_div(st.max_groups, 256)), dim3(256), 0, s,
                       st.d_hi, st.d_off, st.d_gofs, st.max_groups, st.d_planes);
  }
  SCT_LAUNCH_CHECK();
  if (st.timer) st.timer->stop(s, t0, sct::LaunchTimer::BUILD);
  return SCT_OK;
}

int count(State& st, int64_t z_begin, int64_t z_end, unsigned long long* d_counts, hipStream_t s) {
  SCT_CHECK(0 <= z_begin && z_begin <= z_end && z_end <= kSlices, "slice range [%lld, %lld)",
            (long long)z_begin, (long long)z_end);
  if (st.n < 2 || z_begin == z_end) return SCT_OK;
  if (st.lo_bits == kLoBits16) return count16(st, z_begin, z_end, d_counts, s);
  for (int64_t z0 = z_begin; z0 < z_end; z0 += st.chunk) {
    const int z1 = (int)std::min<int64_t>(z_end, z0 + st.chunk);
    // d_counts[0] += n by the job's first tile launch (the range holding slice 0)
    const unsigned long long add_n = z0 == 0 ? (unsigned long long)st.n : 0ull;
    const int rc = st.elem_bytes == 1   ? launch_chunk<int8_t>(st, (int)z0, z1, d_counts, s, add_n)
                   : st.elem_bytes == 2 ? launch_chunk<int16_t>(st, (int)z0, z1, d_counts, s, add_n)
                                        : launch_chunk<int32_t>(st, (int)z0, z1, d_counts, s, add_n);
    if (rc != SCT_OK) return rc;
  }
  return SCT_OK;
}

int time_kernels(State& st, int64_t z_begin, int64_t z_end, unsigned long long* d_counts, int repeats,
                 hipStream_t s, double* seed_ms, double* tile_ms, int64_t* slices) {
  SCT_CHECK(0 <= z_begin && z_begin < z_end && z_end <= kSlices && repeats > 0 && st.n >= 2,
            "time_kernels: empty range or plan");
  if (st.lo_bits == kLoBits16) return time_kernels16(st, z_begin, z_end, d_counts, repeats, s, seed_ms, tile_ms, slices);
  const int z1 = (int)std::min<int64_t>(z_end, z_begin + st.chunk);
  *slices = z1 - z_begin;
  return st.elem_bytes == 1   ? time_chunk<int8_t>(st, (int)z_begin, z1, d_counts, repeats, s, seed_ms, tile_ms)
         : st.elem_bytes == 2 ? time_chunk<int16_t>(st, (int)z_begin, z1, d_counts, repeats, s, seed_ms, tile_ms)
                              : time_chunk<int32_t>(st, (int)z_begin, z1, d_counts, repeats, s, seed_ms, tile_ms);
}

}  // namespace sct_spectral
