// All-pairs TwoBit Hamming-distance histogram for gfx950 (MI355X).
//
// Replaces the O(n^2) pair loop of Barcodes.summarize_hamming_distances
// (src/sctools/barcode.py:42-43), whose per-pair distance is
// TwoBit.hamming_distance (src/sctools/encodings.py:113-121): the number of non-zero
// 2-bit groups of a^b.  The kernel never materialises a distance: it produces, for
// every pair, the distance's bits as bit-planes and counts them.
//
// Data layout
//   codes  : n uint64 TwoBit codes (plan-owned copy), code < 2^(4*NPP).
//   table  : [group pair h][nibble pp < NPP][combo c < 16] -> uint4 {s0_a, s1_a, s0_b, s1_b}
//            for the two 32-code groups a = 2h, b = 2h+1:
//            bit k of s0/s1 = bit 0/1 of  [base_{2pp}(code_{32g+k}) != c&3] +
//                                         [base_{2pp+1}(code_{32g+k}) != c>>2]
//            i.e. for a query whose nibble pp equals c, the 2-bit mismatch count of
//            positions 2pp, 2pp+1 against all 32 codes of the group, bit-sliced.
//            One (h, pp) row is 16 x 16 B = one LDS bank row, so the lanes' ds_read_b128
//            (4 cycles, full LDS rate) never conflict; two groups per read also keeps the
//            compiler from pairing b64 reads into the half-rate ds_read2st64_b64.
//   LDS    : one column chunk = CT groups of the table (32 KiB), resident while a
//            workgroup walks consecutive row blocks of that chunk.
//
// Work decomposition
//   Unordered pairs i<j are covered by items (row block r of RB=256 queries,
//   column chunk c of CB=32*CT codes), enumerated chunk-major: chunk c holds rows
//   r < R(c) = ceil((min((c+1)CB, n) - 1) / RB).  A launch counts any item range
//   [begin, end); each workgroup takes a contiguous sub-range, so it loads a chunk
//   into LDS once and reuses it for every row block of that chunk it visits.
//
// Per (query lane, group of 32 codes):
//   NPP ds_read_b64 select the lane's {s0,s1} planes (the lane's nibble is the LDS
//   offset: no VALU work to form mismatches), a carry-save adder tree of v_bitop3
//   full adders (2 VALU ops each) sums them into B planes d_0..d_{B-1} of the 32
//   distances, and counts[m] += popcount(AND_{b in m} d_b) for m = 1..2*NPP
//   (v_bcnt_u32_b32 accumulates in place).  sct_counts_to_hist inverts the counts.
#include <stdlib.h>

#include <algorithm>
#include <atomic>
#include <vector>

#include <hipcub/hipcub.hpp>

#include "sct_common.h"
#include "spectral.h"

namespace {

constexpr int RB = 256;  // rows (queries) per item == workgroup size

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t maj3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
}

// c += popcount(x) as ONE v_bcnt_u32_b32 (the compiler otherwise re-associates two
// groups' counts into bcnt + bcnt + v_add3, one extra VALU op per pair of counts).
__device__ __forceinline__ void bcnt_acc(uint32_t& c, uint32_t x) {
  asm("v_bcnt_u32_b32 %0, %1, %0" : "+v"(c) : "v"(x));
}

// VGPR banks: a v_bitop3_b32 whose three sources sit in one bank (register index mod 4)
// issues at half rate on gfx950 (profiles/valu_banks_r01.json).  A b128 LDS read lands in
// 4 consecutive registers, so the same component of three reads is three same-bank
// sources -- exactly the adder tree's first level.  The table therefore stores nibble
// pp's four planes rotated by pp mod 4 (slot (k + pp) % 4 holds plane k), which puts the
// planes of consecutive nibbles in consecutive banks; the kernel un-rotates at compile
// time (no instructions).
__host__ __device__ constexpr int plane_slot(int plane, int pp) { return (plane + pp) & 3; }
__device__ __forceinline__ uint32_t comp(const uint4& e, int slot) {
  return slot == 0 ? e.x : (slot == 1 ? e.y : (slot == 2 ? e.z : e.w));
}

constexpr int bitlen(int v) {
  int b = 0;
  while ((1 << b) <= v) ++b;
  return b;
}

// Lookup layout of one group pair (64 codes) in the selection table.
//   nibble layout (SUBSETS): NPP lookups, lookup g = the query's nibble g (bases 2g, 2g+1),
//     16 entries each;
//   triple layout (MOMENTS, 16 bases): 6 lookups -- bases {0,1} and {2,3} (16 entries
//     each) and the triples {4,5,6} {7,8,9} {10,11,12} {13,14,15} (64 entries each): 16
//     2-bit inputs to the adder tree become 6, and with the codes sorted the lanes of a
//     wave share their high bases, so the 64-entry lookups of the high triples broadcast
//     instead of bank-conflicting.
constexpr int kTriNL = 6;
constexpr int kTriRow = 2 * 16 + 4 * 64;  // uint4 entries per group pair
__host__ __device__ constexpr int tri_base(int g) { return g < 2 ? 16 * g : 32 + 64 * (g - 2); }
__host__ __device__ constexpr int tri_shift(int g) { return g < 2 ? 4 * g : 8 + 6 * (g - 2); }
__host__ __device__ constexpr int tri_width(int g) { return g < 2 ? 4 : 6; }

template <int NPP, bool MOM = false>
struct Geom {
  static constexpr int G = 2 * NPP;                  // max distance
  static constexpr int B = MOM ? 4 : bitlen(G);      // distance bit-planes (MOMENTS: d mod 16)
  static constexpr int CT = MOM ? 16 : (NPP <= 8 ? 32 : 16);  // groups per column chunk
  static constexpr int CB = 32 * CT;                 // codes per column chunk
  static constexpr int K = CB / RB;                  // row blocks per chunk step
  static constexpr int NL = MOM ? kTriNL : NPP;      // lookups per group pair
  static constexpr int ROW = MOM ? kTriRow : NPP * 16;  // uint4 entries per group pair
  static constexpr int TILE = CT / 2 * ROW;          // uint4 per chunk (32 / 36 KiB)
};

// LDS offset (uint4 units, within a group-pair row) of lookup g for query q
template <int NPP, bool MOM>
__device__ __forceinline__ int lookup_off(uint64_t q, int g) {
  if constexpr (MOM)
    return tri_base(g) + (int)((q >> tri_shift(g)) & ((1u << tri_width(g)) - 1u));
  else
    return g * 16 + (int)((q >> (4 * g)) & 15u);
}

// Reduce N equal-weight planes to one; writes N/2 carries (next weight).  Balanced
// (Wallace) order: each level compresses every disjoint triple with a full adder in
// parallel, so the dependent depth is ~log_{3/2}(N) levels instead of N/2.  Same
// op count as a linear chain: floor((N-1)/2) full adders + one half adder if N even.
template <int N>
__device__ __forceinline__ uint32_t reduce_col(const uint32_t* in, uint32_t* carry) {
  if constexpr (N == 1) {
    return in[0];
  } else if constexpr (N == 2) {
    carry[0] = in[0] & in[1];
    return in[0] ^ in[1];
  } else {
    constexpr int T = N / 3, R = N % 3;
    uint32_t next[T + R];
#pragma unroll
    for (int t = 0; t < T; ++t) {
      carry[t] = maj3(in[3 * t], in[3 * t + 1], in[3 * t + 2]);
      next[t] = xor3(in[3 * t], in[3 * t + 1], in[3 * t + 2]);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) next[T + r] = in[3 * T + r];
    return reduce_col<T + R>(next, carry + T);
  }
}

template <int W, int N, int B>
__device__ __forceinline__ void reduce_upper(const uint32_t* in, uint32_t (&d)[B]) {
  if constexpr (W < B) {
    if constexpr (N == 0) {
      d[W] = 0;
      reduce_upper<W + 1, 0, B>(in, d);
    } else {
      constexpr int NC = N / 2;
      uint32_t carry[NC > 0 ? NC : 1];
      d[W] = reduce_col<N>(in, carry);
      reduce_upper<W + 1, NC, B>(carry, d);
    }
  }
  // carries beyond plane B-1 are dropped: zero when B = bitlen(2*NPP) (SUBSETS); the
  // MOMENTS scheme drops plane 4 on purpose (B = 4 keeps d mod 16)
}

// Sum NPP 2-bit numbers {s1,s0} into B bit-planes d.
template <int NPP, int B>
__device__ __forceinline__ void adder_tree(const uint32_t (&s0)[NPP], const uint32_t (&s1)[NPP],
                                           uint32_t (&d)[B]) {
  constexpr int C0 = NPP / 2;
  uint32_t c0[C0 > 0 ? C0 : 1];
  d[0] = reduce_col<NPP>(s0, c0);
  constexpr int N1 = NPP + C0;
  uint32_t col1[N1];
#pragma unroll
  for (int k = 0; k < NPP; ++k) col1[k] = s1[k];
#pragma unroll
  for (int k = 0; k < C0; ++k) col1[NPP + k] = c0[k];
  reduce_upper<1, N1, B>(col1, d);
}

// cnt[m-1] += popcount(AND of planes in m), m = 1..G
template <int G, int B>
__device__ __forceinline__ void count_subsets(const uint32_t (&d)[B], uint32_t (&cnt)[G]) {
  uint32_t P[G + 1];
#pragma unroll
  for (int m = 1; m <= G; ++m) {
    const int low = m & (-m);
    const int lb = __builtin_ctz(m);
    const int rest = m ^ low;
    P[m] = rest ? (P[rest] & d[lb]) : d[lb];
    bcnt_acc(cnt[m - 1], P[m]);
  }
}

// MOMENTS scheme: cnt[i] += popcount(AND of the planes in kMomProducts[i]) over the
// four planes of d mod 16 (the d4 carry is never formed).  9 ANDs (three as one
// v_bitop3 3-input AND) + 13 v_bcnt per 32 pairs, against 11 + 16 for count_subsets.
__device__ __forceinline__ uint32_t and3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x80);
}
__device__ __forceinline__ void count_mom(const uint32_t (&d)[4], uint32_t (&cnt)[sct::kMomNProd]) {
  static_assert(sct::kMomNProd == 13, "product list changed: update count_mom");
  const uint32_t p7 = and3(d[0], d[1], d[2]);
  bcnt_acc(cnt[0], d[0]);                    // 1
  bcnt_acc(cnt[1], d[1]);                    // 2
  bcnt_acc(cnt[2], d[0] & d[1]);             // 3
  bcnt_acc(cnt[3], d[2]);                    // 4
  bcnt_acc(cnt[4], d[0] & d[2]);             // 5
  bcnt_acc(cnt[5], d[1] & d[2]);             // 6
  bcnt_acc(cnt[6], p7);                      // 7
  bcnt_acc(cnt[7], d[3]);                    // 8
  bcnt_acc(cnt[8], d[0] & d[3]);             // 9
  bcnt_acc(cnt[9], d[1] & d[3]);             // 10
  bcnt_acc(cnt[10], and3(d[0], d[1], d[3])); // 11
  bcnt_acc(cnt[11], and3(d[0], d[2], d[3])); // 13
  bcnt_acc(cnt[12], p7 & d[3]);              // 15
}

struct ItemCursor {
  int64_t c, r;
};

// items of chunk c (c < nchunks-1): (c+1)*K; prefix P(c) = K*c*(c+1)/2
__device__ __forceinline__ ItemCursor locate_item(int64_t t, int64_t K, int64_t nchunks) {
  double x = sqrt(8.0 * (double)t / (double)K + 1.0);
  int64_t c = (int64_t)((x - 1.0) * 0.5);
  if (c > nchunks - 1) c = nchunks - 1;
  if (c < 0) c = 0;
  while (c > 0 && K * c * (c + 1) / 2 > t) --c;
  while (c < nchunks - 1 && K * (c + 1) * (c + 2) / 2 <= t) ++c;
  return {c, t - K * c * (c + 1) / 2};
}

// valid-pair mask of the 32 codes j0..j0+31 for row i: i < j < n (and i < n)
__device__ __forceinline__ uint32_t pair_mask(int64_t i, int64_t jg, int64_t n) {
  int64_t lo = i + 1 - jg, hi = n - jg;
  lo = lo < 0 ? 0 : (lo > 32 ? 32 : lo);
  hi = hi < 0 ? 0 : (hi > 32 ? 32 : hi);
  uint32_t mask = (uint32_t)(((1ull << hi) - 1ull) & ~((1ull << lo) - 1ull));
  return i < n ? mask : 0u;
}

// counters per lane: SUBSETS 2*NPP subset products, MOMENTS kMomNProd products
template <int NPP, bool MOM>
struct NCount {
  static constexpr int value = MOM ? sct::kMomNProd : 2 * NPP;
};

template <int NPP, bool MASKED, bool MOM, int ABL = 0>
__device__ __forceinline__ void one_group(const uint32_t (&s0)[Geom<NPP, MOM>::NL],
                                          const uint32_t (&s1)[Geom<NPP, MOM>::NL],
                                          int64_t i, int64_t jg, int64_t n,
                                          uint32_t (&cnt)[NCount<NPP, MOM>::value], uint32_t& cnt0) {
  constexpr int NL = Geom<NPP, MOM>::NL;
  constexpr int B = Geom<NPP, MOM>::B;  // MOMENTS: the carry into plane 4 is dropped (d mod 16)
  uint32_t d[B];
  if constexpr (ABL == 4) {  // ablation: no tree and no counting (loads kept live, 1 op each)
#pragma unroll
    for (int b = 0; b < B; ++b) cnt[b] ^= s0[b % NL] ^ s1[(b + 1) % NL];
    return;
  }
  if constexpr (ABL == 2) {  // ablation: no adder tree (planes straight into counting)
#pragma unroll
    for (int b = 0; b < B; ++b) d[b] = s0[b % NL] ^ s1[(b + 1) % NL];
  } else {
    adder_tree<NL, B>(s0, s1, d);
  }
  if constexpr (ABL == 1) {  // ablation: no counting (keep the planes live, 1 op each)
#pragma unroll
    for (int b = 0; b < B; ++b) cnt[b] ^= d[b];
    return;
  }
  if constexpr (MASKED) {
    const uint32_t mask = pair_mask(i, jg, n);
#pragma unroll
    for (int b = 0; b < B; ++b) d[b] &= mask;
    cnt0 += __popc(mask);
  }
  if constexpr (MOM)
    count_mom(d, cnt);
  else
    count_subsets<2 * NPP, B>(d, cnt);
}

template <int NPP, bool MASKED, bool MOM, int UNROLL, int ABL = 0>
__device__ __forceinline__ void process_item(const uint4* __restrict__ tile, uint64_t q, int64_t i,
                                             int64_t j0, int64_t n,
                                             uint32_t (&cnt)[NCount<NPP, MOM>::value],
                                             uint32_t& cnt0) {
  using Gm = Geom<NPP, MOM>;
  constexpr int NL = Gm::NL;
  int off[NL];
#pragma unroll
  for (int g = 0; g < NL; ++g) off[g] = lookup_off<NPP, MOM>(q, g);
  uint4 e0[NL];
  if constexpr (ABL == 3) {  // ablation: no LDS reads after the first group pair
#pragma unroll
    for (int g = 0; g < NL; ++g) e0[g] = tile[off[g]];
  }

  constexpr int U = UNROLL < Gm::CT / 2 ? UNROLL : Gm::CT / 2;
#pragma unroll U
  for (int h = 0; h < Gm::CT / 2; ++h) {
    uint32_t s0a[NL], s1a[NL], s0b[NL], s1b[NL];
#pragma unroll
    for (int g = 0; g < NL; ++g) {
      uint4 e;
      if constexpr (ABL == 3) {
        e = e0[g];
        asm volatile("" : "+v"(e.x), "+v"(e.y), "+v"(e.z), "+v"(e.w));  // opaque: no CSE
      } else {
        e = tile[h * Gm::ROW + off[g]];
      }
      s0a[g] = comp(e, plane_slot(0, g));
      s1a[g] = comp(e, plane_slot(1, g));
      s0b[g] = comp(e, plane_slot(2, g));
      s1b[g] = comp(e, plane_slot(3, g));
    }
    one_group<NPP, MASKED, MOM, ABL>(s0a, s1a, i, j0 + 64 * h, n, cnt, cnt0);
    one_group<NPP, MASKED, MOM, ABL>(s0b, s1b, i, j0 + 64 * h + 32, n, cnt, cnt0);
  }
  if constexpr (!MASKED) cnt0 += Gm::CB;
}

// Count-kernel variants (A/B-selectable with SCT_ALLPAIRS_VARIANT in the ablation build; the
// product build instantiates only the shipped one per scheme): the group-pair loop
// unrolled 1, 2, fully (3: LDS offsets become immediates) or 4 times.  A software-
// pipelined form (next group pair's reads issued before this one's counting) and forced
// occupancy (amdgpu_waves_per_eu) measured no faster and were dropped.
// WAVES > 1 asks the compiler for that many waves per SIMD (amdgpu_waves_per_eu: VGPRs
// capped at 512 / WAVES): variant 5 = unroll 2 held to 128 VGPRs (4 waves per SIMD).
template <int V> struct Variant { static constexpr int UNROLL = V, ABL = 0, WAVES = 1; };
template <> struct Variant<3> { static constexpr int UNROLL = 16, ABL = 0, WAVES = 1; };
#ifdef SCT_ABLATION
template <> struct Variant<5> { static constexpr int UNROLL = 2, ABL = 0, WAVES = 4; };
// ablation builds (wrong results, timing only): 11 no counting, 12 no tree, 13 no LDS reads,
// 14 neither tree nor counting (the loop's fixed costs)
template <> struct Variant<11> { static constexpr int UNROLL = 4, ABL = 1, WAVES = 1; };
template <> struct Variant<12> { static constexpr int UNROLL = 4, ABL = 2, WAVES = 1; };
template <> struct Variant<13> { static constexpr int UNROLL = 4, ABL = 3, WAVES = 1; };
template <> struct Variant<14> { static constexpr int UNROLL = 4, ABL = 4, WAVES = 1; };
#endif

// Workgroup reduction of the per-lane counters: 64-lane butterfly (shfl_xor, lowered to
// DPP/ds_swizzle/ds_bpermute), then LDS across the waves, then one u64 atomic per counter;
// the lane counters restart at 0.  `red` aliases the LDS tile (callers sync first).
template <int G>
__device__ __forceinline__ void flush_counts(uint32_t (&cnt)[G], uint32_t& cnt0,  // G counters
                                             unsigned long long* red,
                                             unsigned long long* __restrict__ out) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  __syncthreads();
#pragma unroll
  for (int m = 0; m <= G; ++m) {
    unsigned long long v = (m == 0) ? cnt0 : cnt[m - 1];
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) v += __shfl_xor(v, s, 64);
    if (lane == 0) red[wave * (G + 1) + m] = v;
  }
  __syncthreads();
  if (tid <= G) {
    unsigned long long s = 0;
#pragma unroll
    for (int w = 0; w < RB / 64; ++w) s += red[w * (G + 1) + tid];
    if (s) atomicAdd(out + tid, s);
  }
#pragma unroll
  for (int m = 0; m < G; ++m) cnt[m] = 0;
  cnt0 = 0;
  __syncthreads();
}

template <int NPP, int V, bool MOM>
__global__ __launch_bounds__(RB) __attribute__((amdgpu_waves_per_eu(Variant<V>::WAVES)))
void allpairs_count_kernel(const uint64_t* __restrict__ codes,
                                                            const uint4* __restrict__ table,
                                                            int64_t n, int64_t nchunks,
                                                            int64_t item_begin, int64_t item_end,
                                                            int64_t grab, int64_t flush_items,
                                                            unsigned long long* __restrict__ queue,
                                                            unsigned long long* __restrict__ out) {
  using Gm = Geom<NPP, MOM>;
  constexpr int G = NCount<NPP, MOM>::value;  // lane counters besides the pair count
  __shared__ __attribute__((aligned(16))) uint4 tile[Gm::TILE];
  __shared__ int64_t s_grab;

  const int tid = threadIdx.x;
  uint32_t cnt[G];
#pragma unroll
  for (int m = 0; m < G; ++m) cnt[m] = 0;
  uint32_t cnt0 = 0;
  const int64_t last_rows = ((n - 1) + RB - 1) / RB;  // R(last chunk)
  int64_t loaded = -1;
  // a lane adds at most CB pairs per item to each u32 counter: flush before 2^32
  // (flush_items <= 0xFFFFFFFF / CB; the host may pass less to exercise the path)
  int64_t since_flush = 0;

  // Dynamic schedule: each workgroup pulls `grab` consecutive items at a time from a
  // device-scope counter (zeroed by a memset node before every launch); consecutive
  // items share a column chunk, so the LDS tile is reloaded only at chunk seams.
  for (;;) {
    __syncthreads();  // everyone is done with s_grab (and, below, with the tile)
    if (tid == 0)
      s_grab = item_begin + (int64_t)__hip_atomic_fetch_add(queue, (unsigned long long)grab,
                                                             __ATOMIC_RELAXED,
                                                             __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int64_t t0 = s_grab;
    if (t0 >= item_end) break;
    const int64_t t1 = t0 + grab < item_end ? t0 + grab : item_end;
    if (since_flush + (t1 - t0) > flush_items) {  // wave-uniform, practically never taken
      flush_counts<G>(cnt, cnt0, reinterpret_cast<unsigned long long*>(tile), out);
      loaded = -1;  // the flush used the tile as scratch
      since_flush = 0;
    }
    since_flush += t1 - t0;
    ItemCursor cur = locate_item(t0, Gm::K, nchunks);
    int64_t i = cur.r * RB + tid;
    uint64_t q = i < n ? codes[i] : 0ull;
    for (int64_t t = t0; t < t1; ++t) {
      const int64_t c = cur.c, r = cur.r;
      if (c != loaded) {
        __syncthreads();  // previous chunk no longer read
        const uint4* src = table + c * Gm::TILE;
#pragma unroll
        for (int k = 0; k < Gm::TILE / RB; ++k) tile[k * RB + tid] = src[k * RB + tid];
        if constexpr (Gm::TILE % RB != 0) {
          const int k = Gm::TILE / RB * RB + tid;
          if (k < Gm::TILE) tile[k] = src[k];
        }
        __syncthreads();
        loaded = c;
      }
      // advance the cursor and prefetch the next item's query while this one computes
      const int64_t rows_c = (c == nchunks - 1) ? last_rows : (c + 1) * Gm::K;
      if (++cur.r >= rows_c) {
        cur.c += 1;
        cur.r = 0;
      }
      const int64_t i_next = cur.r * RB + tid;
      const uint64_t q_next = (t + 1 < t1 && i_next < n) ? codes[i_next] : 0ull;
      const int64_t j0 = c * Gm::CB;
      const bool masked = ((r + 1) * RB > j0) || (j0 + Gm::CB > n);
      if (masked)
        process_item<NPP, true, MOM, Variant<V>::UNROLL, Variant<V>::ABL>(tile, q, i, j0, n, cnt,
                                                                          cnt0);
      else
        process_item<NPP, false, MOM, Variant<V>::UNROLL, Variant<V>::ABL>(tile, q, i, j0, n, cnt,
                                                                           cnt0);
      q = q_next;
      i = i_next;
    }
  }

  flush_counts<G>(cnt, cnt0, reinterpret_cast<unsigned long long*>(tile), out);
}

// table[h][pp][c] = bit-sliced 2-bit mismatch counts of nibble pp of the 64 codes of
// group pair h against combo c (see file header).  One thread per entry.
__global__ void allpairs_build_kernel(const uint64_t* __restrict__ codes, int64_t n, int npp,
                                      int64_t e_begin, int64_t e_end, uint4* __restrict__ table) {
  const int64_t idx = e_begin + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= e_end) return;
  const int c = (int)(idx & 15);
  const int pp = (int)((idx >> 4) % npp);
  const int64_t h = (idx >> 4) / npp;
  uint32_t s[4] = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int half = 0; half < 2; ++half) {
#pragma unroll 8
    for (int k = 0; k < 32; ++k) {
      const int64_t j = h * 64 + half * 32 + k;
      const uint64_t code = j < n ? codes[j] : 0ull;
      const uint32_t x = (uint32_t)((code >> (4 * pp)) & 15u) ^ (uint32_t)c;
      const uint32_t m0 = (x & 3u) != 0u, m1 = (x >> 2) != 0u;
      s[2 * half] |= (m0 ^ m1) << k;
      s[2 * half + 1] |= (m0 & m1) << k;
    }
  }
  uint32_t r[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) r[plane_slot(k, pp)] = s[k];
  table[idx] = make_uint4(r[0], r[1], r[2], r[3]);
}

// Triple layout (MOMENTS): entry (h, lookup g, value c) = bit-sliced mismatch counts
// (0..3) of the bases of lookup g of the 64 codes of group pair h against the query's
// bases c.  A workgroup builds 4 group pairs: each wave transposes its 64 codes into
// base bit-planes with 32 ballots (lane k = code k, so ballot = both groups' planes),
// then every thread forms entries from the planes held in LDS: per base, mismatch =
// (lo ^ c_lo) | (hi ^ c_hi), and the 2-3 mismatch planes are summed by a half/full adder.
__global__ __launch_bounds__(256) void allpairs_build_tri_kernel(const uint64_t* __restrict__ codes,
                                                                 int64_t n, int64_t gp_begin,
                                                                 int64_t gp_end,
                                                                 uint4* __restrict__ table) {
  __shared__ uint64_t planes[4][32];  // [wave][2 * base + bit], group a = low 32 bits
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t h0 = gp_begin + (int64_t)blockIdx.x * 4;
  {
    const int64_t j = (h0 + wave) * 64 + lane;
    const uint32_t code = j < n ? (uint32_t)codes[j] : 0u;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      const uint64_t b = __ballot((code >> k) & 1u);
      if (lane == k) planes[wave][k] = b;
    }
  }
  __syncthreads();
  const int64_t nh = gp_end - h0 < 4 ? gp_end - h0 : 4;
  for (int t = threadIdx.x; t < nh * kTriRow; t += 256) {
    const int w = t / kTriRow, e = t - w * kTriRow;
    const int g = e < 32 ? (e >> 4) : 2 + ((e - 32) >> 6);
    const uint32_t c = (uint32_t)(e - tri_base(g));
    const int base0 = tri_shift(g) / 2, nb = tri_width(g) / 2;
    uint64_t mm[3];
    for (int k = 0; k < 3; ++k) {
      if (k < nb) {
        const uint64_t lo = planes[w][2 * (base0 + k)], hi = planes[w][2 * (base0 + k) + 1];
        const uint32_t d = (c >> (2 * k)) & 3u;
        mm[k] = (lo ^ ((d & 1u) ? ~0ull : 0ull)) | (hi ^ ((d & 2u) ? ~0ull : 0ull));
      } else {
        mm[k] = 0ull;
      }
    }
    const uint64_t s0 = mm[0] ^ mm[1] ^ mm[2];
    const uint64_t s1 = (mm[0] & mm[1]) | (mm[2] & (mm[0] ^ mm[1]));
    const uint32_t sv[4] = {(uint32_t)s0, (uint32_t)s1, (uint32_t)(s0 >> 32), (uint32_t)(s1 >> 32)};
    uint32_t r[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) r[plane_slot(k, g)] = sv[k];
    table[(h0 + w) * kTriRow + e] = make_uint4(r[0], r[1], r[2], r[3]);
  }
}

// ---------------------------------------------------------------- agreement moments
// M_k = #(pair, k-set of positions S) with the pair agreeing on all of S
//     = sum over pairs of C(16 - d, k) = sum_{|S|=k} sum_{pattern} C(count_S(pattern), 2),
// k = 1..3.  Only the 3-position marginals are counted (560 position triples x 64
// patterns = 35,840 bins); the 2- and 1-position marginals are sums of triple bins.
// No atomics: the codes are first transposed into position/base bitmasks
//   masks[w][4p + a] bit k = [base p of code 32w + k == a]            (moments_masks_kernel)
// and every marginal bin is a popcount of an AND of three of them
//   count(p,a, q,b, r,c) = sum_w popcount(masks[w][4p+a] & masks[w][4q+b] & masks[w][4r+c])
// (moments_count_kernel: a workgroup stages kMomWR words of masks in LDS; each thread
// owns one triple and one base b of its middle position and sweeps all words, 16
// bitop3 + 16 v_bcnt per word for its 16 bins).  Partial bins per word range are summed
// by moments_reduce_kernel; moments_finalize_kernel turns bins into C(count, 2).
constexpr int kMomWR = 256;     // mask words (8,192 codes) per LDS range: 64 KiB
constexpr int kMomTri = 64;     // triples per workgroup (4 threads each)
constexpr int kMomNTri = 560;   // C(16, 3)
constexpr int kMomNPair = 120;  // C(16, 2)

struct MomTriple {
  uint32_t shifts;  // p | q << 8 | r << 16, p < q < r (base positions)
};

// marginal of a pair/single read off one triple: the triple, and the slot(s) kept
struct MomSource {
  int32_t tri;
  int32_t slot;  // pair: the free slot (summed); single: the kept slot
};

// one wave per 64 codes (= 2 mask words): lane l builds masks[.][l] from 64 ballots
__global__ __launch_bounds__(256) void moments_masks_kernel(const uint64_t* __restrict__ codes,
                                                            int64_t n, int64_t nwords,
                                                            uint32_t* __restrict__ masks) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int64_t w0 = wave * 2;
  if (w0 >= nwords) return;
  const int64_t i = w0 * 32 + lane;
  const bool valid = i < n;
  const uint32_t c = valid ? (uint32_t)codes[i] : 0u;
  uint32_t lo = 0, hi = 0;
#pragma unroll
  for (int pa = 0; pa < 64; ++pa) {
    const uint64_t b = __ballot(valid && ((c >> (2 * (pa >> 2))) & 3u) == (uint32_t)(pa & 3));
    if (lane == pa) {
      lo = (uint32_t)b;
      hi = (uint32_t)(b >> 32);
    }
  }
  masks[w0 * 64 + lane] = lo;
  if (w0 + 1 < nwords) masks[(w0 + 1) * 64 + lane] = hi;
}

// grid (word ranges, triple blocks); partial[range][tri * 64 + (a << 4 | b << 2 | c)]
__global__ __launch_bounds__(256) void moments_count_kernel(const uint32_t* __restrict__ masks,
                                                            int64_t nwords,
                                                            const MomTriple* __restrict__ tri,
                                                            int tri0, int tri1,
                                                            uint32_t* __restrict__ partial) {
  __shared__ __attribute__((aligned(16))) uint32_t m[kMomWR * 64];
  const int64_t wbeg = (int64_t)blockIdx.x * kMomWR;
  const int nw = (int)min<int64_t>(kMomWR, nwords - wbeg);
  {
    const uint4* src = reinterpret_cast<const uint4*>(masks + wbeg * 64);
    uint4* dst = reinterpret_cast<uint4*>(m);
    for (int k = threadIdx.x; k < nw * 16; k += 256) dst[k] = src[k];
  }
  __syncthreads();
  const int t = tri0 + blockIdx.y * kMomTri + (threadIdx.x >> 2);
  if (t >= tri1) return;
  const int b = threadIdx.x & 3;
  const uint32_t sh = tri[t].shifts;
  const int p = sh & 255, q = (sh >> 8) & 255, r = (sh >> 16) & 255;
  uint32_t cnt[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) cnt[k] = 0u;
  const uint4* m4 = reinterpret_cast<const uint4*>(m);
  for (int w = 0; w < nw; ++w) {
    const uint4 P = m4[w * 16 + p];
    const uint4 R = m4[w * 16 + r];
    const uint32_t Q = m[w * 64 + 4 * q + b];
    const uint32_t pa[4] = {P.x, P.y, P.z, P.w};
    const uint32_t rc[4] = {R.x, R.y, R.z, R.w};
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int c = 0; c < 4; ++c) bcnt_acc(cnt[a * 4 + c], and3(pa[a], Q, rc[c]));
  }
  uint32_t* out = partial + (int64_t)blockIdx.x * kMomNTri * 64 + (int64_t)t * 64;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c) out[(a << 4) | (b << 2) | c] = cnt[a * 4 + c];
}

// ghist[bin] = sum over word ranges of partial[range][bin], bins [b0, b1)
__global__ __launch_bounds__(256) void moments_reduce_kernel(const uint32_t* __restrict__ partial,
                                                             int nranges, int b0, int b1,
                                                             unsigned* __restrict__ ghist) {
  const int k = b0 + blockIdx.x * 256 + threadIdx.x;
  if (k >= b1) return;
  unsigned s = 0;
  for (int rg = 0; rg < nranges; ++rg) s += partial[(int64_t)rg * kMomNTri * 64 + k];
  ghist[k] = s;
}

__device__ __forceinline__ unsigned long long pairs_of(unsigned long long c) {
  return c * (c - (c > 0ull)) / 2ull;
}

// Triples [tri0, tri1) are complete in ghist.  Adds to out[0..2] (M1, M2, M3):
//   M3 += C(bin, 2) over those triples' bins;
//   M2 += C(pair bin, 2) for the pairs whose source triple lies in the range (4-bin sums);
//   M1 += C(single bin, 2) likewise (16-bin sums).
__global__ __launch_bounds__(256) void moments_finalize_kernel(const unsigned* __restrict__ ghist,
                                                               int tri0, int tri1,
                                                               const MomSource* __restrict__ pair_src,
                                                               const MomSource* __restrict__ single_src,
                                                               unsigned long long* __restrict__ out) {
  unsigned long long acc[3] = {0ull, 0ull, 0ull};
  const int nb3 = (tri1 - tri0) * 64;
  const int total = nb3 + kMomNPair * 16 + sct::kMomG * 4;
  for (int k = blockIdx.x * 256 + threadIdx.x; k < total; k += gridDim.x * 256) {
    if (k < nb3) {
      acc[2] += pairs_of(ghist[(int64_t)tri0 * 64 + k]);
    } else if (k < nb3 + kMomNPair * 16) {
      const int j = k - nb3, pr = j >> 4, ab = j & 15;
      const MomSource src = pair_src[pr];
      if (src.tri < tri0 || src.tri >= tri1) continue;
      // kept slots in order, free slot f: bin = digits (slot0, slot1, slot2), 2 bits each
      const int f = src.slot;
      unsigned long long c = 0;
      for (int v = 0; v < 4; ++v) {
        int dig[3], kk = 0;
        for (int sl = 0; sl < 3; ++sl) dig[sl] = (sl == f) ? v : ((kk++ == 0) ? (ab >> 2) : (ab & 3));
        c += ghist[(int64_t)src.tri * 64 + (dig[0] << 4) + (dig[1] << 2) + dig[2]];
      }
      acc[1] += pairs_of(c);
    } else {
      const int j = k - nb3 - kMomNPair * 16, p = j >> 2, a = j & 3;
      const MomSource src = single_src[p];
      if (src.tri < tri0 || src.tri >= tri1) continue;
      unsigned long long c = 0;
      for (int v = 0; v < 16; ++v) {
        int dig[3], kk = 0;
        for (int sl = 0; sl < 3; ++sl) dig[sl] = (sl == src.slot) ? a : ((kk++ == 0) ? (v >> 2) : (v & 3));
        c += ghist[(int64_t)src.tri * 64 + (dig[0] << 4) + (dig[1] << 2) + dig[2]];
      }
      acc[0] += pairs_of(c);
    }
  }
  __shared__ unsigned long long red[3][4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int o = 0; o < 3; ++o) {
    unsigned long long v = acc[o];
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) v += __shfl_xor(v, s, 64);
    if (lane == 0) red[o][wave] = v;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    const unsigned long long v = red[threadIdx.x][0] + red[threadIdx.x][1] + red[threadIdx.x][2] +
                                 red[threadIdx.x][3];
    if (v) atomicAdd(out + threadIdx.x, v);
  }
}

// groups per column chunk: nibble layout 32 (16 above 8 nibbles), triple layout 16
int ct_for(int npp, bool tri) { return tri ? 16 : (npp <= 8 ? 32 : 16); }
bool mom_supported(int npp, int64_t n) { return npp * 2 == sct::kMomG && n <= 100000000LL; }
// SPECTRAL: the same 16-base codes; its cost does not depend on n
bool spectral_supported(int npp, int64_t n) { return mom_supported(npp, n); }
// smallest n for which AUTO picks SPECTRAL over MOMENTS (measured crossover)
int64_t spectral_min_n() { return sct::tune(SCT_TUNE_SPECTRAL_MIN_N, 325000); }
// what SCT_ALLPAIRS_AUTO resolves to
int auto_scheme(int npp, int64_t n) {
  if (spectral_supported(npp, n) && n >= spectral_min_n()) return SCT_ALLPAIRS_SPECTRAL;
  return mom_supported(npp, n) ? SCT_ALLPAIRS_MOMENTS : SCT_ALLPAIRS_SUBSETS;
}
bool auto_moments(int npp, int64_t n) { return auto_scheme(npp, n) == SCT_ALLPAIRS_MOMENTS; }

}  // namespace

struct sct_allpairs_plan {
  int device = 0;
  int64_t n = 0;
  int code_bits = 0;
  int npp = 0;
  int nbins = 0;
  int ct = 0;
  int64_t cb = 0;
  int64_t nchunks = 0;
  int64_t items = 0;
  int grid = 0;
  uint64_t* d_codes = nullptr;
  uint64_t* d_sorted = nullptr;  // MOMENTS: the codes sorted (rows of a wave share high bases)
  void* d_sort_tmp = nullptr;
  size_t sort_tmp_bytes = 0;
  uint4* d_table = nullptr;
  int64_t table_entries = 0;
  int variant = 2;  // count-kernel variant (SCT_ALLPAIRS_VARIANT=1..4, see Variant<>)
  int64_t grab = 16;  // items per work-queue pull (SCT_ALLPAIRS_GRAB)
  int64_t flush_items = 0;  // test hook: flush lane counters more often (SCT_ALLPAIRS_FLUSH_ITEMS)
  unsigned long long* d_queue = nullptr;  // work-queue head, zeroed before every launch
  int scheme = SCT_ALLPAIRS_SUBSETS;
  int ncounts = 0;
  // MOMENTS scheme: position triples, pair/single sources, and the global triple bins
  MomTriple* d_mtri = nullptr;
  MomSource* d_msrc = nullptr;  // kMomNPair pair sources, then kMomG single sources
  unsigned* d_mhist = nullptr;
  uint32_t* d_mmasks = nullptr;    // [nwords][64] position/base bitmasks
  uint32_t* d_mpartial = nullptr;  // [nranges][560 * 64] partial bins
  int64_t mom_nwords = 0;
  int mom_nranges = 0;
  sct_spectral::State spec;  // SPECTRAL scheme (spectral.hip)
  sct::LaunchTimer timer;    // bench aid (sct_allpairs_timing)
};

namespace {

int64_t rows_of_chunk(const sct_allpairs_plan* p, int64_t c) {
  const int64_t maxj = std::min<int64_t>((c + 1) * p->cb, p->n) - 1;
  return maxj <= 0 ? 0 : (maxj + RB - 1) / RB;
}

// The count kernel instantiations a plan can launch: (variant, scheme) -> kernel.
// SUBSETS: variants 1, 2 (and 3 = full unroll at 16 bases); MOMENTS (16 bases only):
// 1, 2, 3, 4; ablation builds add 11..13 at 16 bases.
template <int NPP>
struct CountKernels {
  using Fn = void (*)(const uint64_t*, const uint4*, int64_t, int64_t, int64_t, int64_t, int64_t,
                      int64_t, unsigned long long*, unsigned long long*);
  static Fn get(int variant, int scheme) {
#ifdef SCT_ABLATION
    if constexpr (NPP == 8) {
      if (scheme == SCT_ALLPAIRS_MOMENTS) {
        switch (variant) {
          case 1: return allpairs_count_kernel<NPP, 1, true>;
          case 3: return allpairs_count_kernel<NPP, 3, true>;
          case 4: return allpairs_count_kernel<NPP, 4, true>;
          case 5: return allpairs_count_kernel<NPP, 5, true>;
          case 11: return allpairs_count_kernel<NPP, 11, true>;
          case 12: return allpairs_count_kernel<NPP, 12, true>;
          case 13: return allpairs_count_kernel<NPP, 13, true>;
          case 14: return allpairs_count_kernel<NPP, 14, true>;
          default: return allpairs_count_kernel<NPP, 2, true>;
        }
      }
      switch (variant) {
        case 1: return allpairs_count_kernel<NPP, 1, false>;
        case 3: return allpairs_count_kernel<NPP, 3, false>;
        case 11: return allpairs_count_kernel<NPP, 11, false>;
        case 12: return allpairs_count_kernel<NPP, 12, false>;
        case 13: return allpairs_count_kernel<NPP, 13, false>;
        default: return allpairs_count_kernel<NPP, 2, false>;
      }
    } else {
      if (scheme == SCT_ALLPAIRS_MOMENTS) return nullptr;
      return variant == 1 ? allpairs_count_kernel<NPP, 1, false> : allpairs_count_kernel<NPP, 2, false>;
    }
#else
    // the shipped variants: MOMENTS unroll 1, SUBSETS at 16 bases full
    // unroll, SUBSETS at other widths unroll 2
    (void)variant;
    if constexpr (NPP == 8) {
      if (scheme == SCT_ALLPAIRS_MOMENTS) return allpairs_count_kernel<NPP, 1, true>;
      return allpairs_count_kernel<NPP, 3, false>;
    } else {
      if (scheme == SCT_ALLPAIRS_MOMENTS) return nullptr;
      return allpairs_count_kernel<NPP, 2, false>;
    }
#endif
  }
};

template <int NPP>
int launch_count(sct_allpairs_plan* p, int64_t b, int64_t e, uint64_t* d_counts, int grid,
                 hipStream_t s) {
  auto fn = CountKernels<NPP>::get(p->variant, p->scheme);
  if (!fn) return sct::fail(SCT_E_INVALID, "MOMENTS scheme needs 16-base codes");
  if (grid <= 0) grid = p->grid;
  const int64_t total = e - b;
  if (grid > total) grid = (int)total;
  SCT_CHECK(p->grab > 0 && p->grab * p->cb < 0xFFFFFFFFLL, "grab too large");
  // a lane adds at most cb pairs per item to each u32 counter: flush before 2^32
  int64_t flush = 0xFFFFFFFFLL / p->cb - p->grab;
  if (p->flush_items > 0 && p->flush_items < flush) flush = p->flush_items;
  SCT_HIP(hipMemsetAsync(p->d_queue, 0, sizeof(unsigned long long), s));
  const uint64_t* codes = p->d_sorted ? p->d_sorted : p->d_codes;
  hipEvent_t t0 = p->timer.start(s);
  hipLaunchKernelGGL(fn, dim3(grid), dim3(RB), 0, s, codes, p->d_table, p->n, p->nchunks, b, e,
                     p->grab, flush, p->d_queue, reinterpret_cast<unsigned long long*>(d_counts));
  SCT_LAUNCH_CHECK();
  p->timer.stop(s, t0, sct::LaunchTimer::COUNT);
  return SCT_OK;
}

template <int NPP>
int occupancy_grid(int cus, int variant, int scheme) {
  int per_cu = 0;
  auto fn = CountKernels<NPP>::get(variant, scheme);
  if (!fn || hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, RB, 0) != hipSuccess ||
      per_cu <= 0)
    per_cu = 4;
  return cus * per_cu;  // persistent: every workgroup resident, pulling from the queue
}

#define SCT_NPP_SWITCH(npp, FN, ...)     \
  switch (npp) {                         \
    case 1: return FN<1>(__VA_ARGS__);   \
    case 2: return FN<2>(__VA_ARGS__);   \
    case 3: return FN<3>(__VA_ARGS__);   \
    case 4: return FN<4>(__VA_ARGS__);   \
    case 5: return FN<5>(__VA_ARGS__);   \
    case 6: return FN<6>(__VA_ARGS__);   \
    case 7: return FN<7>(__VA_ARGS__);   \
    case 8: return FN<8>(__VA_ARGS__);   \
    case 9: return FN<9>(__VA_ARGS__);   \
    case 10: return FN<10>(__VA_ARGS__); \
    case 11: return FN<11>(__VA_ARGS__); \
    case 12: return FN<12>(__VA_ARGS__); \
    case 13: return FN<13>(__VA_ARGS__); \
    case 14: return FN<14>(__VA_ARGS__); \
    case 15: return FN<15>(__VA_ARGS__); \
    case 16: return FN<16>(__VA_ARGS__); \
    default: break;                      \
  }

int grid_for(int npp, int cus, int variant, int scheme) {
  SCT_NPP_SWITCH(npp, occupancy_grid, cus, variant, scheme);
  return cus * 4;
}

int dispatch_count(sct_allpairs_plan* p, int64_t b, int64_t e, uint64_t* d, int grid,
                   hipStream_t s) {
  SCT_NPP_SWITCH(p->npp, launch_count, p, b, e, d, grid, s);
  return sct::fail(SCT_E_RANGE, "unsupported npp %d", p->npp);
}

// The 560 position triples p < q < r (lexicographic), and for every pair / single the
// triple its marginal is read from: pair (p,q) -> (p,q,r) with r the smallest other
// position (slot of r summed); single p -> (p,q,r) with q, r the two smallest others.
void mom_layout(std::vector<MomTriple>& tri, std::vector<MomSource>& src) {
  static_assert(sct::kMomOrder == 3, "moment layout assumes order 3");
  tri.clear();
  src.clear();
  int index[16][16][16];
  for (int p = 0; p < sct::kMomG; ++p)
    for (int q = p + 1; q < sct::kMomG; ++q)
      for (int r = q + 1; r < sct::kMomG; ++r) {
        index[p][q][r] = (int)tri.size();
        tri.push_back(MomTriple{(uint32_t)p | (uint32_t)q << 8 | (uint32_t)r << 16});
      }
  auto sorted_source = [&](int a, int b, int c, int special) {
    int v[3] = {a, b, c};
    std::sort(v, v + 3);
    const int slot = v[0] == special ? 0 : (v[1] == special ? 1 : 2);
    return MomSource{index[v[0]][v[1]][v[2]], slot};
  };
  for (int p = 0; p < sct::kMomG; ++p)
    for (int q = p + 1; q < sct::kMomG; ++q) {
      int r = 0;
      while (r == p || r == q) ++r;
      src.push_back(sorted_source(p, q, r, r));  // free slot = r's
    }
  for (int p = 0; p < sct::kMomG; ++p) {
    int o[2], k = 0;
    for (int x = 0; x < sct::kMomG && k < 2; ++x)
      if (x != p) o[k++] = x;
    src.push_back(sorted_source(p, o[0], o[1], p));  // kept slot = p's
  }
}

}  // namespace

extern "C" int sct_allpairs_plan_create(const uint64_t* d_codes, int64_t n, int code_bits,
                                        sct_allpairs_plan** plan) {
  return sct_allpairs_plan_create_ex(d_codes, n, code_bits, SCT_ALLPAIRS_AUTO, plan);
}

extern "C" int sct_allpairs_plan_create_ex(const uint64_t* d_codes, int64_t n, int code_bits,
                                           int scheme, sct_allpairs_plan** plan) {
  return sct_allpairs_plan_create_ex2(d_codes, n, code_bits, scheme, 0, plan);
}

extern "C" int sct_allpairs_plan_create_ex2(const uint64_t* d_codes, int64_t n, int code_bits, int scheme,
                                            int flags, sct_allpairs_plan** plan) {
  SCT_CHECK(plan != nullptr, "plan is NULL");
  SCT_CHECK((flags & ~(SCT_ALLPAIRS_DISTINCT | SCT_ALLPAIRS_NO_CACHE)) == 0, "unknown plan flags 0x%x", flags);
  SCT_CHECK(scheme == SCT_ALLPAIRS_AUTO || scheme == SCT_ALLPAIRS_SUBSETS ||
                scheme == SCT_ALLPAIRS_MOMENTS || scheme == SCT_ALLPAIRS_SPECTRAL,
            "unknown scheme %d", scheme);
  *plan = nullptr;
  SCT_CHECK(n >= 0, "n must be >= 0");
  SCT_CHECK(n == 0 || d_codes != nullptr, "codes is NULL");
  SCT_CHECK(code_bits <= 64, "code_bits %d > 64: codes wider than 64 bits are not supported",
            code_bits);
  // SPECTRAL slices per seed / tile pass: all 2^18 (one 4 GiB intermediate) for cached plans; a
  // plan mapping its own memory (the one-shot drop-in call) maps a 1 GiB intermediate and makes
  // four passes: 3.26 / 4.71 / 4.06 ms per config-2 drop-in call against 3.50 / 4.79 / 4.53 for
  // one pass, three rounds on one box (tools/dropin_chunk_ab.py, profiles/ab_dropin_chunk_r06b.jsonl)
  const int64_t chunk_knob = sct::tune(SCT_TUNE_SPECTRAL_CHUNK, (flags & SCT_ALLPAIRS_NO_CACHE) ? 65536 : 262144);
  auto* p = new sct_allpairs_plan();
  auto cleanup = [&](int rc) {
    sct_allpairs_plan_destroy(p);
    return rc;
  };
  hipError_t e = hipGetDevice(&p->device);
  if (e != hipSuccess) return cleanup(sct::fail(SCT_E_HIP, "hipGetDevice: %s", hipGetErrorString(e)));
  p->n = n;
  // the device's cached buffers (plan cache, spectral.h) when no other plan holds them
  if (flags & SCT_ALLPAIRS_NO_CACHE) {
    // the plan's own buffers, carved from one block: the codes, the probe's scratch and (for a
    // set AUTO sends to SPECTRAL) the transform's buffers with its 4 GiB intermediate
    size_t est = ((size_t)n * 8 + 255) + ((size_t)36 << 20);
    if (n >= 2 && n >= sct::tune(SCT_TUNE_SPECTRAL_MIN_N, 325000)) {
      // the intermediate: one chunk of 16-KiB slices (int8, 14-bit columns; a set dense enough for
      // 16-bit columns maps the rest of its larger intermediate separately)
      const int64_t chunk = std::min<int64_t>(std::max<int64_t>(chunk_knob, 64), 262144);
      est += (size_t)n * 4 + ((size_t)n / 32 + 65536) * 80 + (size_t)((chunk + 15) & ~15ll) * 16384 + ((size_t)16 << 20);
    }
    p->spec.ws = sct_spectral::ws_arena(est);
  } else {
    p->spec.ws = sct_spectral::ws_acquire();
  }
  // one probe of the codes: their OR (code width) and the densest transform columns (SPECTRAL's
  // seed width), one synchronisation
  unsigned long long probe[3] = {0, 0, 0};
  if (n > 0) {
    void* dc = nullptr;
    if (int rc = sct_spectral::ws_get(p->spec.ws, sct_spectral::W_CODES, (size_t)n * 8, &dc); rc != SCT_OK)
      return cleanup(rc);
    p->d_codes = reinterpret_cast<uint64_t*>(dc);
    e = hipMemcpyAsync(p->d_codes, d_codes, (size_t)n * 8, hipMemcpyDefault, 0);
    if (e != hipSuccess) return cleanup(sct::fail(SCT_E_HIP, "copy codes: %s", hipGetErrorString(e)));
    if (int rc = sct_spectral::probe(p->spec.ws, p->d_codes, n, probe); rc != SCT_OK) return cleanup(rc);
  }
  const unsigned long long orv = probe[0];
  int need = 0;
  while (need < 64 && (orv >> need)) ++need;
  if (code_bits <= 0) code_bits = need;
  if (need > code_bits)
    return cleanup(sct::fail(SCT_E_RANGE, "a code needs %d bits but code_bits=%d", need, code_bits));
  if (code_bits < 1) code_bits = 1;
  p->code_bits = code_bits;
  p->npp = (code_bits + 3) / 4;
  p->nbins = 2 * p->npp + 1;
  // MOMENTS needs 16-base codes (29..32 bits); AUTO picks it there
  // (u32 marginal bins and u64 M_3 <= C(n,2)*560 bound n; 1e8 codes is far beyond a whitelist)
  const bool mom_ok = mom_supported(p->npp, n);
  if (scheme == SCT_ALLPAIRS_MOMENTS && !mom_ok)
    return cleanup(sct::fail(SCT_E_INVALID, "MOMENTS scheme needs code_bits in 29..32 (got %d) "
                             "and n <= 1e8", code_bits));
  if (scheme == SCT_ALLPAIRS_SPECTRAL && !spectral_supported(p->npp, n))
    return cleanup(sct::fail(SCT_E_INVALID, "SPECTRAL scheme needs code_bits in 29..32 (got %d) "
                             "and n <= 1e8", code_bits));
  p->scheme = scheme == SCT_ALLPAIRS_AUTO ? auto_scheme(p->npp, n) : scheme;
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, p->device) != hipSuccess ||
      cus <= 0)
    cus = 256;
  if (p->scheme == SCT_ALLPAIRS_SPECTRAL) {
    // items = the 4096 transform slices; no selection table
    p->ncounts = sct_spectral::kNCounts;
    p->items = n >= 2 ? sct_spectral::kSlices : 0;
    p->spec.distinct = (flags & SCT_ALLPAIRS_DISTINCT) != 0;
    const int rc = sct_spectral::create(p->spec, p->d_codes, n, chunk_knob, cus,
                                        (unsigned)probe[1], (unsigned)probe[2]);
    if (rc != SCT_OK) return cleanup(rc);
    p->spec.timer = &p->timer;
    *plan = p;
    return SCT_OK;
  }
  p->ncounts = p->scheme == SCT_ALLPAIRS_MOMENTS ? sct::kMomNCounts : p->nbins;
  const bool tri = p->scheme == SCT_ALLPAIRS_MOMENTS;
  p->ct = ct_for(p->npp, tri);
  p->cb = 32LL * p->ct;
  p->nchunks = n > 0 ? sct::ceil_div(n, p->cb) : 0;
  p->items = 0;
  if (n >= 2) {
    const int64_t K = p->cb / RB;
    const int64_t last = p->nchunks - 1;
    p->items = K * last * (last + 1) / 2 + rows_of_chunk(p, last);
  }
  p->table_entries = p->nchunks * (p->ct / 2) * (int64_t)(tri ? kTriRow : p->npp * 16);
  if (p->table_entries > 0) {
    e = hipMalloc(&p->d_table, (size_t)p->table_entries * sizeof(uint4));
    if (e != hipSuccess) return cleanup(sct::fail(SCT_E_NOMEM, "hipMalloc table: %s", hipGetErrorString(e)));
  }
  e = hipMalloc(&p->d_queue, sizeof(unsigned long long));
  if (e != hipSuccess) return cleanup(sct::fail(SCT_E_NOMEM, "hipMalloc queue: %s", hipGetErrorString(e)));
  if (tri && n > 0) {
    // sorted row order: the lanes of a wave then share their high bases
    e = hipMalloc(&p->d_sorted, (size_t)n * 8);
    if (e == hipSuccess)
      e = hipcub::DeviceRadixSort::SortKeys(nullptr, p->sort_tmp_bytes, (const uint64_t*)nullptr,
                                            (uint64_t*)nullptr, (int)n, 0, 32);
    if (e == hipSuccess) e = hipMalloc(&p->d_sort_tmp, std::max<size_t>(p->sort_tmp_bytes, 16));
    if (e != hipSuccess) return cleanup(sct::fail(SCT_E_NOMEM, "sort buffers: %s", hipGetErrorString(e)));
  }
  if (p->scheme == SCT_ALLPAIRS_MOMENTS) {
    std::vector<MomTriple> tri;
    std::vector<MomSource> src;
    mom_layout(tri, src);
    e = hipMalloc(&p->d_mtri, tri.size() * sizeof(MomTriple));
    if (e == hipSuccess) e = hipMalloc(&p->d_msrc, src.size() * sizeof(MomSource));
    if (e == hipSuccess) e = hipMalloc(&p->d_mhist, (size_t)kMomNTri * 64 * sizeof(unsigned));
    p->mom_nwords = sct::ceil_div(std::max<int64_t>(n, 1), 32);
    p->mom_nranges = (int)sct::ceil_div(p->mom_nwords, kMomWR);
    if (e == hipSuccess) e = hipMalloc(&p->d_mmasks, (size_t)(p->mom_nwords + 1) * 64 * sizeof(uint32_t));
    if (e == hipSuccess)
      e = hipMalloc(&p->d_mpartial, (size_t)p->mom_nranges * kMomNTri * 64 * sizeof(uint32_t));
    if (e != hipSuccess) return cleanup(sct::fail(SCT_E_NOMEM, "hipMalloc moments: %s", hipGetErrorString(e)));
    e = hipMemcpy(p->d_mtri, tri.data(), tri.size() * sizeof(MomTriple), hipMemcpyHostToDevice);
    if (e == hipSuccess)
      e = hipMemcpy(p->d_msrc, src.data(), src.size() * sizeof(MomSource), hipMemcpyHostToDevice);
    if (e != hipSuccess) return cleanup(sct::fail(SCT_E_HIP, "copy moments layout: %s", hipGetErrorString(e)));
  }
  // defaults measured on MI355X: MOMENTS unroll 1, SUBSETS@16 bases full unroll
  p->variant = p->scheme == SCT_ALLPAIRS_MOMENTS ? 1 : (p->npp == 8 ? 3 : 2);
  // MOMENTS: 32 items per pull halves the chunk re-staging (L2 -> LDS) at no cost in time
  if (p->scheme == SCT_ALLPAIRS_MOMENTS) p->grab = 32;
#ifdef SCT_ABLATION
  // timing-only build: count-kernel ablations 11..14 (wrong results by design)
  if (const char* v = getenv("SCT_ALLPAIRS_VARIANT")) {
    const int vv = atoi(v);
    if ((vv >= 1 && vv <= 3) || ((vv == 4 || vv == 5) && p->scheme == SCT_ALLPAIRS_MOMENTS) ||
        (vv >= 11 && vv <= 14))
      p->variant = vv;
  }
#endif
  p->grid = grid_for(p->npp, cus, p->variant, p->scheme);
  p->flush_items = sct::tune(SCT_TUNE_ALLPAIRS_FLUSH_ITEMS, 0);
  if (const int64_t g = sct::tune(SCT_TUNE_ALLPAIRS_GRAB, 0); g > 0) p->grab = g;
  if (const int64_t g = sct::tune(SCT_TUNE_ALLPAIRS_GRID, 0); g > 0) p->grid = (int)g;
  *plan = p;
  return SCT_OK;
}

extern "C" int sct_allpairs_plan_destroy(sct_allpairs_plan* plan) {
  if (!plan) return SCT_OK;
  sct_spectral::wait_idle(plan->spec);  // (every scheme's work is recorded there) before any buffer goes
  if (plan->d_codes) sct_spectral::ws_put(plan->spec.ws, plan->d_codes);  // (the workspace: kept)
  if (plan->d_sorted) (void)hipFree(plan->d_sorted);
  if (plan->d_sort_tmp) (void)hipFree(plan->d_sort_tmp);
  if (plan->d_table) (void)hipFree(plan->d_table);
  if (plan->d_queue) (void)hipFree(plan->d_queue);
  if (plan->d_mtri) (void)hipFree(plan->d_mtri);
  if (plan->d_msrc) (void)hipFree(plan->d_msrc);
  if (plan->d_mhist) (void)hipFree(plan->d_mhist);
  if (plan->d_mmasks) (void)hipFree(plan->d_mmasks);
  if (plan->d_mpartial) (void)hipFree(plan->d_mpartial);
  sct_spectral::destroy(plan->spec);
  delete plan;
  return SCT_OK;
}

extern "C" int sct_allpairs_plan_info(const sct_allpairs_plan* plan, int* nbins, int64_t* items,
                                      int64_t* pairs) {
  SCT_CHECK(plan != nullptr, "plan is NULL");
  if (nbins) *nbins = plan->nbins;
  if (items) *items = plan->items;
  if (pairs) *pairs = plan->n * (plan->n - 1) / 2;
  return SCT_OK;
}

extern "C" int sct_allpairs_plan_scheme(const sct_allpairs_plan* plan, int* scheme, int* ncounts,
                                        int* code_bits) {
  SCT_CHECK(plan != nullptr, "plan is NULL");
  if (scheme) *scheme = plan->scheme;
  if (ncounts) *ncounts = plan->ncounts;
  if (code_bits) *code_bits = plan->code_bits;
  return SCT_OK;
}

extern "C" int sct_allpairs_moments(sct_allpairs_plan* plan, int part, int nparts,
                                    uint64_t* d_counts, void* stream) {
  SCT_CHECK(plan != nullptr, "plan is NULL");
  SCT_CHECK(nparts >= 1 && 0 <= part && part < nparts, "part %d of %d", part, nparts);
  if (plan->scheme != SCT_ALLPAIRS_MOMENTS || plan->n < 2) return SCT_OK;
  SCT_CHECK(d_counts != nullptr, "counts is NULL");
  // part p histograms triples [560p/P, 560(p+1)/P) and owns the pairs/singles read off them
  const int t0 = (int)((int64_t)kMomNTri * part / nparts);
  const int t1 = (int)((int64_t)kMomNTri * (part + 1) / nparts);
  if (t0 == t1) return SCT_OK;
  hipStream_t s = sct::as_stream(stream);
  const int64_t nwaves = sct::ceil_div(plan->mom_nwords, 2);
  hipLaunchKernelGGL(moments_masks_kernel, dim3((unsigned)sct::ceil_div(nwaves, 4)), dim3(256), 0, s,
                     plan->d_codes, plan->n, plan->mom_nwords, plan->d_mmasks);
  SCT_LAUNCH_CHECK();
  hipLaunchKernelGGL(moments_count_kernel, dim3(plan->mom_nranges, (unsigned)sct::ceil_div(t1 - t0, kMomTri)),
                     dim3(256), 0, s, plan->d_mmasks, plan->mom_nwords, plan->d_mtri, t0, t1,
                     plan->d_mpartial);
  SCT_LAUNCH_CHECK();
  hipLaunchKernelGGL(moments_reduce_kernel, dim3((unsigned)sct::ceil_div((t1 - t0) * 64, 256)), dim3(256), 0,
                     s, plan->d_mpartial, plan->mom_nranges, t0 * 64, t1 * 64, plan->d_mhist);
  SCT_LAUNCH_CHECK();
  const int work = (t1 - t0) * 64 + kMomNPair * 16 + sct::kMomG * 4;
  const int fblocks = (int)std::min<int64_t>(160, sct::ceil_div(work, 256));
  hipLaunchKernelGGL(moments_finalize_kernel, dim3(fblocks), dim3(256), 0, s, plan->d_mhist, t0, t1,
                     plan->d_msrc, plan->d_msrc + kMomNPair,
                     reinterpret_cast<unsigned long long*>(d_counts) + 1 + sct::kMomNProd);
  SCT_LAUNCH_CHECK();
  sct_spectral::note_stream(plan->spec, s);
  return SCT_OK;
}

namespace {
// column chunk holding work item t (items are chunk-major, chunk c has rows_of_chunk(c))
int64_t chunk_of_item(const sct_allpairs_plan* p, int64_t t) {
  int64_t c = 0, base = 0;
  while (c < p->nchunks - 1 && base + rows_of_chunk(p, c) <= t) base += rows_of_chunk(p, c++);
  return c;
}
}  // namespace

extern "C" int sct_allpairs_build(sct_allpairs_plan* plan, void* stream) {
  SCT_CHECK(plan != nullptr, "plan is NULL");
  return sct_allpairs_build_items(plan, 0, plan->items, stream);
}

extern "C" int sct_allpairs_build_items(sct_allpairs_plan* plan, int64_t item_begin, int64_t item_end,
                                        void* stream) {
  SCT_CHECK(plan != nullptr, "plan is NULL");
  SCT_CHECK(0 <= item_begin && item_begin <= item_end && item_end <= plan->items,
            "item range [%lld, %lld) outside [0, %lld)", (long long)item_begin, (long long)item_end,
            (long long)plan->items);
  hipStream_t s = sct::as_stream(stream);
  if (plan->scheme == SCT_ALLPAIRS_SPECTRAL) {
    const int rc = sct_spectral::build(plan->spec, plan->d_codes, s);
    sct_spectral::note_stream(plan->spec, s);
    return rc;
  }
  if (plan->table_entries == 0) return SCT_OK;
  // only the column chunks the items read (a rank of a sharded job builds its own slice)
  int64_t c0 = 0, c1 = plan->nchunks;
  if (item_end > item_begin) {
    c0 = chunk_of_item(plan, item_begin);
    c1 = chunk_of_item(plan, item_end - 1) + 1;
  } else {
    c1 = 0;
  }
  const int64_t gp_per_chunk = plan->ct / 2;
  hipEvent_t t0 = plan->timer.start(s);
  if (plan->scheme == SCT_ALLPAIRS_MOMENTS) {
    // every row block may be read: the whole (sorted) code list is needed
    size_t bytes = plan->sort_tmp_bytes;
    SCT_HIP(hipcub::DeviceRadixSort::SortKeys(plan->d_sort_tmp, bytes, (const uint64_t*)plan->d_codes,
                                              plan->d_sorted, (int)plan->n, 0, 32, s));
    const int64_t gp0 = c0 * gp_per_chunk, ngp = (c1 - c0) * gp_per_chunk;
    if (ngp > 0)
      hipLaunchKernelGGL(allpairs_build_tri_kernel, dim3((unsigned)sct::ceil_div(ngp, 4)), dim3(256), 0,
                         s, plan->d_sorted, plan->n, gp0, gp0 + ngp, plan->d_table);
  } else {
    const int64_t row = (int64_t)plan->npp * 16;
    const int64_t e0 = c0 * gp_per_chunk * row, e1 = c1 * gp_per_chunk * row;
    if (e1 > e0)
      hipLaunchKernelGGL(allpairs_build_kernel, dim3((unsigned)sct::ceil_div(e1 - e0, 256)), dim3(256), 0,
                         s, plan->d_codes, plan->n, plan->npp, e0, e1, plan->d_table);
  }
  SCT_LAUNCH_CHECK();
  plan->timer.stop(s, t0, sct::LaunchTimer::BUILD);
  sct_spectral::note_stream(plan->spec, s);
  return SCT_OK;
}

extern "C" int sct_allpairs_spectral_info(const sct_allpairs_plan* plan, int* elem_bytes, int64_t* chunk_slices,
                                          int* max_column) {
  SCT_CHECK(plan != nullptr, "plan is NULL");
  SCT_CHECK(plan->scheme == SCT_ALLPAIRS_SPECTRAL, "not a SPECTRAL plan");
  if (elem_bytes) *elem_bytes = plan->spec.elem_bytes;
  if (chunk_slices) *chunk_slices = plan->spec.chunk;
  if (max_column) *max_column = (int)plan->spec.max_m;
  return SCT_OK;
}

extern "C" int sct_allpairs_spectral_columns(const sct_allpairs_plan* plan, int* column_bits) {
  SCT_CHECK(plan != nullptr && column_bits != nullptr, "NULL pointer");
  SCT_CHECK(plan->scheme == SCT_ALLPAIRS_SPECTRAL, "not a SPECTRAL plan");
  *column_bits = plan->spec.lo_bits;
  return SCT_OK;
}

extern "C" int sct_allpairs_timing(sct_allpairs_plan* plan, int mode, double* out) {
  SCT_CHECK(plan != nullptr, "plan is NULL");
  SCT_CHECK(mode >= 0 && mode <= 2, "mode %d: 0 stop, 1 start, 2 read", mode);
  sct::LaunchTimer& t = plan->timer;
  if (mode == 1) {
    t.reset();
    t.on = true;
  } else {
    t.collect();
    if (mode == 0) t.on = false;
  }
  if (out)
    for (int k = 0; k < sct::LaunchTimer::NKINDS; ++k) {
      out[2 * k] = t.ms[k];
      out[2 * k + 1] = (double)t.launches[k];
    }
  return SCT_OK;
}

extern "C" int sct_allpairs_count(sct_allpairs_plan* plan, int64_t item_begin, int64_t item_end,
                                  uint64_t* d_counts, int grid, void* stream) {
  SCT_CHECK(plan != nullptr, "plan is NULL");
  sct::scalar_quiesce();  // persistent grids below size themselves to the resident slots
  SCT_CHECK(d_counts != nullptr, "counts is NULL");
  SCT_CHECK(0 <= item_begin && item_begin <= item_end && item_end <= plan->items,
            "item range [%lld, %lld) outside [0, %lld)", (long long)item_begin,
            (long long)item_end, (long long)plan->items);
  if (item_begin == item_end) return SCT_OK;
  hipStream_t s = sct::as_stream(stream);
  const int rc = plan->scheme == SCT_ALLPAIRS_SPECTRAL
                     ? sct_spectral::count(plan->spec, item_begin, item_end,
                                           reinterpret_cast<unsigned long long*>(d_counts), s)
                     : dispatch_count(plan, item_begin, item_end, d_counts, grid, s);
  sct_spectral::note_stream(plan->spec, s);
  return rc;
}

extern "C" int sct_allpairs_time_kernels(sct_allpairs_plan* plan, int64_t item_begin, int64_t item_end,
                                         uint64_t* d_counts, int repeats, double* out, void* stream) {
  sct::scalar_quiesce();
  SCT_CHECK(plan != nullptr && d_counts != nullptr && out != nullptr, "NULL pointer");
  SCT_CHECK(0 <= item_begin && item_begin < item_end && item_end <= plan->items && repeats > 0,
            "item range [%lld, %lld) outside [0, %lld) or repeats < 1", (long long)item_begin,
            (long long)item_end, (long long)plan->items);
  hipStream_t s = sct::as_stream(stream);
  sct_spectral::note_stream(plan->spec, s);  // (the call synchronises before it returns)
  if (plan->scheme == SCT_ALLPAIRS_SPECTRAL) {
    int64_t slices = 0;
    const int rc = sct_spectral::time_kernels(plan->spec, item_begin, item_end,
                                              reinterpret_cast<unsigned long long*>(d_counts), repeats, s,
                                              &out[1], &out[0], &slices);
    out[2] = (double)slices;
    return rc;
  }
  hipEvent_t e[2];
  SCT_HIP(hipEventCreate(&e[0]));
  SCT_HIP(hipEventCreate(&e[1]));
  int rc = SCT_OK;
  (void)hipEventRecord(e[0], s);
  for (int r = 0; rc == SCT_OK && r < repeats; ++r) rc = dispatch_count(plan, item_begin, item_end, d_counts, 0, s);
  (void)hipEventRecord(e[1], s);
  float ms = 0;
  if (rc == SCT_OK && hipEventSynchronize(e[1]) == hipSuccess) (void)hipEventElapsedTime(&ms, e[0], e[1]);
  (void)hipEventDestroy(e[0]);
  (void)hipEventDestroy(e[1]);
  out[0] = ms / repeats;
  out[1] = 0;
  out[2] = (double)(item_end - item_begin);
  return rc;
}

extern "C" int sct_allpairs_geometry(int64_t n, int code_bits, int* nbins, int64_t* items,
                                     int* rows_per_item, int* cols_per_item) {
  SCT_CHECK(n >= 0, "n must be >= 0");
  SCT_CHECK(code_bits >= 1 && code_bits <= 64, "code_bits %d outside [1, 64]", code_bits);
  const int npp = (code_bits + 3) / 4;
  if (auto_scheme(npp, n) == SCT_ALLPAIRS_SPECTRAL) {  // items = transform slices
    if (nbins) *nbins = 2 * npp + 1;
    if (items) *items = n >= 2 ? sct_spectral::kSlices : 0;
    if (rows_per_item) *rows_per_item = 0;
    if (cols_per_item) *cols_per_item = 0;
    return SCT_OK;
  }
  const int64_t cb = 32LL * ct_for(npp, auto_moments(npp, n));
  const int64_t nchunks = n > 0 ? sct::ceil_div(n, cb) : 0;
  int64_t it = 0;
  if (n >= 2) {
    const int64_t K = cb / RB, last = nchunks - 1;
    const int64_t maxj = std::min<int64_t>((last + 1) * cb, n) - 1;
    it = K * last * (last + 1) / 2 + (maxj <= 0 ? 0 : (maxj + RB - 1) / RB);
  }
  if (nbins) *nbins = 2 * npp + 1;
  if (items) *items = it;
  if (rows_per_item) *rows_per_item = RB;
  if (cols_per_item) *cols_per_item = (int)cb;
  return SCT_OK;
}

extern "C" int sct_allpairs_range_pairs(const sct_allpairs_plan* plan, int64_t item_begin,
                                        int64_t item_end, int64_t* pairs) {
  SCT_CHECK(plan != nullptr && pairs != nullptr, "NULL pointer");
  SCT_CHECK(0 <= item_begin && item_begin <= item_end && item_end <= plan->items,
            "item range outside the plan");
  const int64_t n = plan->n;
  if (plan->scheme == SCT_ALLPAIRS_SPECTRAL) {
    // pairs are not split by slice: a slice range is credited its share of all pairs,
    // floor(P * end / items) - floor(P * begin / items), which sums to P over a partition
    const __int128 P = (__int128)n * (n - 1) / 2;
    *pairs = plan->items ? (int64_t)(P * item_end / plan->items - P * item_begin / plan->items) : 0;
    return SCT_OK;
  }
  int64_t total = 0, c = 0, base = 0;
  while (c < plan->nchunks && base + rows_of_chunk(plan, c) <= item_begin) base += rows_of_chunk(plan, c++);
  int64_t r = item_begin - base;
  for (int64_t t = item_begin; t < item_end; ++t) {
    // pairs of item (c, r) = #{(i, j): i in row block r, j in chunk c, i < j < n}
    const int64_t jlo = c * plan->cb, jhi = std::min<int64_t>((c + 1) * plan->cb, n);
    const int64_t ilo = r * RB, ihi = std::min<int64_t>((r + 1) * RB, n);
    const int64_t a_hi = std::min(ihi, jlo);  // rows i < jlo see the whole chunk
    if (a_hi > ilo) total += (a_hi - ilo) * (jhi - jlo);
    const int64_t b_lo = std::max(ilo, jlo), b_hi = std::min(ihi, jhi - 1);  // i in chunk: jhi-1-i
    if (b_hi > b_lo) total += (b_hi - b_lo) * (2 * jhi - 1 - b_lo - b_hi) / 2;
    if (++r >= rows_of_chunk(plan, c)) {
      ++c;
      r = 0;
    }
  }
  *pairs = total;
  return SCT_OK;
}

extern "C" int sct_hamming_hist_allpairs_host(const uint64_t* codes, int64_t n, int code_bits,
                                              uint64_t* hist, int nbins) {
  return sct_hamming_hist_allpairs_host_ex(codes, n, code_bits, 0, hist, nbins);
}

namespace {
// one device's share of a one-shot all-pairs job (sct_hamming_hist_allpairs_host*): a plan on the
// current device over the n host codes, built, then moment part `part` of `nparts` and item range
// items * part / nparts .. items * (part + 1) / nparts counted; the raw counts come back to `counts`
// (129 words) with the plan's scheme / counts length / bins.  Without the keep-workspace setting
// (sct_keep_workspace) every device buffer of the call is its own and freed before it returns.
struct Share {
  uint64_t counts[129] = {};
  int scheme = 0, ncounts = 0, nbins = 0;
};
std::atomic<int> g_keep_ws{0};

int allpairs_share_host(const uint64_t* codes, int64_t n, int code_bits, int flags, int part, int nparts,
                        Share* out) {
  const bool keep = g_keep_ws.load(std::memory_order_relaxed) != 0;
  // codes and counts: the thread's cached staging buffer when the workspace is kept (no per-call
  // hipMalloc), else a buffer of the call's own
  const size_t cbytes = ((size_t)n * 8 + 255) & ~(size_t)255, need = cbytes + 129 * 8;
  sct::DevBuf own;
  uint8_t* base = nullptr;
  if (keep) {
    sct::HostStage* hs = sct::host_stage();
    if (!hs) return SCT_E_HIP;
    if (int rc = sct::stage_reserve(hs, 0, need); rc != SCT_OK) return rc;
    base = hs->dev;
  } else {
    SCT_HIP(own.alloc(need));
    base = static_cast<uint8_t*>(own.p);
  }
  uint64_t* d_codes = reinterpret_cast<uint64_t*>(base);
  uint64_t* d_counts = reinterpret_cast<uint64_t*>(base + cbytes);
  if (n) SCT_HIP(hipMemcpyAsync(d_codes, codes, (size_t)n * 8, hipMemcpyHostToDevice, 0));
  sct_allpairs_plan* plan = nullptr;
  int rc = sct_allpairs_plan_create_ex2(d_codes, n, code_bits, SCT_ALLPAIRS_AUTO,
                                        flags | (keep ? 0 : SCT_ALLPAIRS_NO_CACHE), &plan);
  if (rc != SCT_OK) return rc;
  struct Guard {
    sct_allpairs_plan* p;
    ~Guard() { sct_allpairs_plan_destroy(p); }  // (waits for the plan's work: before `own` is freed)
  } guard{plan};
  out->scheme = plan->scheme;
  out->ncounts = plan->ncounts;
  out->nbins = plan->nbins;
  const int64_t b = plan->items * part / nparts, e = plan->items * (part + 1) / nparts;
  SCT_HIP(hipMemsetAsync(d_counts, 0, (size_t)plan->ncounts * 8, 0));
  rc = sct_allpairs_build_items(plan, b, e, nullptr);
  if (rc != SCT_OK) return rc;
  rc = sct_allpairs_moments(plan, part, nparts, d_counts, nullptr);
  if (rc != SCT_OK) return rc;
  rc = sct_allpairs_count(plan, b, e, d_counts, 0, nullptr);
  if (rc != SCT_OK) return rc;
  SCT_HIP(hipMemcpy(out->counts, d_counts, (size_t)plan->ncounts * 8, hipMemcpyDeviceToHost));
  return SCT_OK;
}

// the shares' counts summed (mod 2^64, as an int64 all-reduce sums them), checked and inverted
int allpairs_finish(const Share* sh, int nshares, int64_t n, uint64_t* hist, int nbins) {
  uint64_t counts[129] = {};
  for (int r = 0; r < nshares; ++r) {
    if (sh[r].scheme != sh[0].scheme || sh[r].ncounts != sh[0].ncounts || sh[r].nbins != sh[0].nbins)
      return sct::fail(SCT_E_HIP, "device shares disagree on the plan (scheme %d / %d)", sh[0].scheme, sh[r].scheme);
    for (int k = 0; k < sh[r].ncounts; ++k) counts[k] += sh[r].counts[k];
  }
  if (sh[0].nbins != nbins) return sct::fail(SCT_E_INVALID, "hist holds %d bins, plan needs %d", nbins, sh[0].nbins);
  // counts[0]: pairs counted (SUBSETS, MOMENTS) or the code count (SPECTRAL)
  const int64_t expect = sh[0].scheme == SCT_ALLPAIRS_SPECTRAL ? n : n * (n - 1) / 2;
  if ((int64_t)counts[0] != (n >= 2 ? expect : 0))
    return sct::fail(SCT_E_HIP, "pair count mismatch: counted %llu, expected %lld", (unsigned long long)counts[0],
                     (long long)expect);
  return sct_counts_to_hist_ex(sh[0].scheme, counts, sh[0].ncounts, hist, nbins);
}
}  // namespace

extern "C" int sct_hamming_hist_allpairs_host_ex(const uint64_t* codes, int64_t n, int code_bits, int flags,
                                                 uint64_t* hist, int nbins) {
  SCT_CHECK(hist != nullptr, "hist is NULL");
  SCT_CHECK(n >= 0 && (n == 0 || codes != nullptr), "bad codes");
  SCT_CHECK((flags & ~SCT_ALLPAIRS_DISTINCT) == 0, "unknown flags 0x%x", flags);
  Share sh;
  if (int rc = allpairs_share_host(codes, n, code_bits, flags, 0, 1, &sh); rc != SCT_OK) return rc;
  return allpairs_finish(&sh, 1, n, hist, nbins);
}

extern "C" int sct_hamming_hist_allpairs_host_devices(const uint64_t* codes, int64_t n, int code_bits, int flags,
                                                      const int* devices, int ndev, uint64_t* hist, int nbins) {
  SCT_CHECK(hist != nullptr, "hist is NULL");
  SCT_CHECK(n >= 0 && (n == 0 || codes != nullptr), "bad codes");
  SCT_CHECK((flags & ~SCT_ALLPAIRS_DISTINCT) == 0, "unknown flags 0x%x", flags);
  std::vector<Share> sh((size_t)std::max(ndev, 1));
  const int rc = sct::run_on_devices(devices, ndev, [&](int r) {
    return allpairs_share_host(codes, n, code_bits, flags, r, ndev, &sh[(size_t)r]);
  });
  if (rc != SCT_OK) return rc;
  return allpairs_finish(sh.data(), ndev, n, hist, nbins);
}

extern "C" int sct_keep_workspace(int keep, int* previous) {
  const int was = g_keep_ws.load();
  if (previous) *previous = was;
  if (keep >= 0) g_keep_ws.store(keep ? 1 : 0);
  return SCT_OK;
}

extern "C" int sct_allpairs_cache_release(void) {
  sct_spectral::ws_release_all();
  (void)hipDeviceSynchronize();  // (the stream-ordered frees have completed)
  sct::pool_trim();
  sct::stage_release_device();
  return SCT_OK;
}
