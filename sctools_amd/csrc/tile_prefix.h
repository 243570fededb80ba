// Tile prefixes without a scan and without a look-back chain (round 4).  A count pass writes
// every tile's count and last position; tile_sums_reduce_kernel (one wave per 1,024 tiles) sums
// them into two coarser levels (blocks of 32 and of 1,024 tiles); a later pass gets tile t's
// exclusive prefix from at most (t >> 10) + 31 + 31 of those values, which the workgroup's
// threads load at once.  Measured instead: a decoupled look-back inside one pass (whitelist
// 1.37 ms, FASTQ 18.8 ms: on MI355X a cross-CU hand-off costs ~1 us, MI355X_MICROARCH.md handoff
// rows, and a tile looks back over the ~1,500 tiles in flight) and the count pass adding into the
// coarse levels with atomics (whitelist count pass 147 us for 62.7 MB: every tile in flight adds
// to the same one or two words).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sct {

// l values are "position + 1" (0 = none)
struct TileSums {
  unsigned long long* c0;  // [ntiles] count of tile t (written by its count workgroup)
  unsigned long long* c1;  // [ceil(ntiles / 32)] sums over blocks of 32 tiles (tile_sums_reduce_kernel)
  unsigned long long* c2;  // [ceil(ntiles / 1024)] sums over blocks of 1024 tiles
  unsigned long long* l0;  // nullable: [ntiles] last position + 1 of tile t, 0 if none
  unsigned long long* l1;  // maxima over blocks of 32
  unsigned long long* l2;  // maxima over blocks of 1024
  uint32_t* f0;            // nullable: [ntiles] flags of tile t (written by its count workgroup)
  uint32_t* fany;          // with f0: the OR of every f0 (zeroed by the count pass's workgroup 0)
};

// bytes of the scratch for ntiles tiles: c0 | l0 | c1 | c2 | l1 | l2 (| f0 | fany)
inline size_t tile_sums_bytes(int64_t ntiles, bool with_flags = false) {
  const size_t n1 = (size_t)((ntiles + 31) >> 5), n2 = (size_t)((ntiles + 1023) >> 10);
  return 16 * ((size_t)ntiles + n1 + n2) + (with_flags ? 4 * (size_t)ntiles + 8 : 0);
}
inline TileSums tile_sums_at(void* base, int64_t ntiles, bool with_last, bool with_flags = false) {
  unsigned long long* p = reinterpret_cast<unsigned long long*>(base);
  const int64_t n1 = (ntiles + 31) >> 5, n2 = (ntiles + 1023) >> 10;
  TileSums s;
  s.c0 = p;
  s.l0 = with_last ? p + ntiles : nullptr;
  s.c1 = p + 2 * ntiles;
  s.c2 = s.c1 + n1;
  s.l1 = s.c2 + n2;
  s.l2 = s.l1 + n1;
  s.f0 = with_flags ? reinterpret_cast<uint32_t*>(s.l2 + n2) : nullptr;
  s.fany = with_flags ? s.f0 + ntiles : nullptr;
  return s;
}

// one thread per tile: publish tile t's count and last position (-1: none)
__device__ __forceinline__ void tile_publish(const TileSums& s, int64_t t, unsigned long long cnt, long long last) {
  s.c0[t] = cnt;
  if (s.l0) s.l0[t] = (unsigned long long)(last + 1);
}

// one 64-lane wave per 1,024 tiles: lane i sums tiles [16 i, 16 i + 16) of the block, lane pairs
// form the 32-tile sums, the wave the 1,024-tile sum (launch ceil(ntiles / 1024) blocks of 64).
// skip / skip_gen: as the count passes' spec_fail / spec_gen -- when a one-read pass ran and did
// the whole job (*skip != skip_gen) the count pass wrote nothing, so there is nothing to reduce
static __global__ __launch_bounds__(64) void tile_sums_reduce_kernel(TileSums s, int64_t ntiles,
                                                                     const unsigned* skip = nullptr,
                                                                     unsigned skip_gen = 0) {
  if (skip && *skip != skip_gen) return;
  const int lane = threadIdx.x;
  const int64_t t0 = (int64_t)blockIdx.x * 1024 + 16 * lane;
  unsigned long long c = 0, l = 0;
  for (int k = 0; k < 16; ++k)
    if (t0 + k < ntiles) {
      c += s.c0[t0 + k];
      if (s.l0) l = l > s.l0[t0 + k] ? l : s.l0[t0 + k];
    }
  const unsigned long long c2 = c + __shfl_xor(c, 1), lo = __shfl_xor(l, 1), l2 = l > lo ? l : lo;
  if (!(lane & 1) && t0 < ntiles) {
    s.c1[(t0 >> 5)] = c2;
    if (s.l0) s.l1[(t0 >> 5)] = l2;
  }
  unsigned long long cs = c, ls = l;
#pragma unroll
  for (int o = 32; o; o >>= 1) {
    cs += __shfl_xor(cs, o);
    const unsigned long long m = __shfl_xor(ls, o);
    ls = ls > m ? ls : m;
  }
  if (lane == 0) {
    s.c2[blockIdx.x] = cs;
    if (s.l0) s.l2[blockIdx.x] = ls;
  }
  if (s.f0) {  // the OR of the tile flags: an atomic only from a block that has one set
    uint32_t f = 0;
    for (int k = 0; k < 16; ++k)
      if (t0 + k < ntiles) f |= s.f0[t0 + k];
#pragma unroll
    for (int o = 32; o; o >>= 1) f |= __shfl_xor(f, o);
    if (lane == 0 && f) atomicOr(s.fany, f);
  }
}

// every thread of a WG-thread workgroup: tile t's exclusive count and the last position before it
// (-1: none) into *cnt / *last (shared), and with total != nullptr the count over all tiles (the
// n2 = ceil(ntiles / 1024) block sums); one barrier inside, one at the end
template <int WG>
__device__ __forceinline__ void tile_prefix(const TileSums& s, int64_t t, unsigned long long* cnt, long long* last,
                                            unsigned long long (*red)[WG / 64], int64_t n2 = 0,
                                            unsigned long long* total = nullptr) {
  const int64_t A = t >> 10, B = (t >> 5) & 31, C = t & 31, N = A + B + C + (total ? n2 : 0);
  unsigned long long sum = 0, mx = 0, all = 0;
  for (int64_t j = threadIdx.x; j < N; j += WG) {
    if (j >= A + B + C) {
      all += s.c2[j - A - B - C];
      continue;
    }
    const unsigned long long* cp;
    const unsigned long long* lq;
    int64_t k;
    if (j < A) {
      cp = s.c2;
      lq = s.l2;
      k = j;
    } else if (j < A + B) {
      cp = s.c1;
      lq = s.l1;
      k = (t >> 10) * 32 + (j - A);
    } else {
      cp = s.c0;
      lq = s.l0;
      k = (t >> 5) * 32 + (j - A - B);
    }
    sum += cp[k];
    if (s.l0) mx = mx > lq[k] ? mx : lq[k];
  }
#pragma unroll
  for (int o = 32; o; o >>= 1) {
    sum += __shfl_xor(sum, o);
    all += __shfl_xor(all, o);
    const unsigned long long m2 = __shfl_xor(mx, o);
    mx = mx > m2 ? mx : m2;
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][wave] = sum;
    red[1][wave] = mx;
    red[2][wave] = all;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long a = 0, b = 0, c = 0;
    for (int w = 0; w < WG / 64; ++w) {
      a += red[0][w];
      b = b > red[1][w] ? b : red[1][w];
      c += red[2][w];
    }
    *cnt = a;
    *last = (long long)b - 1;
    if (total) *total = c;
  }
  __syncthreads();
}

// Without the coarse levels (small buffers: ntiles up to a few thousand): every thread of the
// workgroup sums tile t's exclusive count and the last position before it straight from c0 / l0,
// and ORs every tile's flag (f0, nullable) -- ntiles / WG loads per thread, no reduction launch.
template <int WG>
__device__ __forceinline__ void tile_prefix_direct(const TileSums& s, int64_t t, int64_t ntiles, unsigned long long* cnt,
                                                   long long* last, uint32_t* flags_any,
                                                   unsigned long long (*red)[WG / 64]) {
  unsigned long long sum = 0, mx = 0, fl = 0;
  for (int64_t k = threadIdx.x; k < ntiles; k += WG) {
    if (k < t) {
      sum += s.c0[k];
      if (s.l0) mx = mx > s.l0[k] ? mx : s.l0[k];
    }
    if (s.f0) fl |= s.f0[k];
  }
#pragma unroll
  for (int o = 32; o; o >>= 1) {
    sum += __shfl_xor(sum, o);
    fl |= __shfl_xor(fl, o);
    const unsigned long long m2 = __shfl_xor(mx, o);
    mx = mx > m2 ? mx : m2;
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][wave] = sum;
    red[1][wave] = mx;
    red[2][wave] = fl;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long a = 0, b = 0, c = 0;
    for (int w = 0; w < WG / 64; ++w) {
      a += red[0][w];
      b = b > red[1][w] ? b : red[1][w];
      c |= red[2][w];
    }
    *cnt = a;
    *last = (long long)b - 1;
    *flags_any = (uint32_t)c;
  }
  __syncthreads();
}

}  // namespace sct
