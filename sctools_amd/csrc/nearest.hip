// Nearest-whitelist correction on gfx950 (config 4).
//
// There is no reference function for this.  The contract is the
// brute-force composition of the reference's distance (TwoBit.hamming_distance,
// encodings.py:113-121, or ThreeBit.hamming_distance, encodings.py:194-202): for each
// query q, d_min = min_j dist(q, w_j);
//   index[q] = j   if d_min <= max_d and exactly one whitelist index j attains it,
//            = -2  if d_min <= max_d and two or more indices attain it (tie),
//            = -1  if d_min > max_d;
//   dist[q]  = d_min if d_min <= max_d else 255.
//
// Algorithm (exact pigeonhole index): split the G base positions into P = max_d + 1
// contiguous blocks; any w with dist(q, w) <= max_d agrees with q exactly on at least
// one block.  For each block the whitelist is bucketed by a multiplicative hash of that
// block's bits into ~4x as many buckets as the block has distinct values (CSR: u32
// offsets[b] .. offsets[b+1] into 8-byte code entries + a 4-byte index array read only for
// candidates; built by a histogram / exclusive-scan / scatter on the GPU).  A query issues
// all P bucket-offset loads before it reads any entry (one dependent random access per
// probe; the offset tables are sized to stay in each XCD's L2), then
// verifies every entry of its P buckets with the full distance, so hash collisions never
// change the result.  A code found through several blocks has one index, so it is never
// counted as a tie with itself.
#include <hipcub/hipcub.hpp>

#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>

#include "sct_common.h"

namespace {

constexpr int WG = 256;
constexpr int MAX_PARTS = 8;

struct Part {
  uint64_t mask;  // the block's bits, in place
  uint64_t mul;   // multiplicative hash (0 when there is a single bucket)
  int lo_bit;     // first bit of the block in the code
  int nbits;      // bits of the block (<= 64)
  int shift;      // 64 - log2(buckets), in [1, 63]
};

// branch-free (uniform branches would split the probes' loads into separate waits)
__device__ __forceinline__ uint32_t part_bucket(uint64_t code, Part p) {
  return (uint32_t)((((code & p.mask) >> p.lo_bit) * p.mul) >> p.shift);
}

__device__ __forceinline__ int dist2(uint64_t a, uint64_t b) {
  const uint64_t x = a ^ b;
  return __popcll((x | (x >> 1)) & 0x5555555555555555ull);
}
__device__ __forceinline__ int dist3(uint64_t a, uint64_t b) {
  const uint64_t x = a ^ b;
  return __popcll((x | (x >> 1) | (x >> 2)) & 0x9249249249249249ull);
}

struct Parts {
  Part p[MAX_PARTS];
};

__global__ void key_hist_kernel(const uint64_t* __restrict__ wl, int64_t nw, Part part,
                                uint32_t* __restrict__ counts) {
  for (int64_t j = (int64_t)blockIdx.x * WG + threadIdx.x; j < nw; j += (int64_t)gridDim.x * WG)
    atomicAdd(&counts[part_bucket(wl[j], part)], 1u);
}

// entries: codes[pos] (8 B, what a probe scans) and index[pos] (read only for a new best);
// index bit 31 = the code occurs more than once in the whitelist (flag_dups_kernel)
__global__ void key_scatter_kernel(const uint64_t* __restrict__ wl, int64_t nw, Part part,
                                   uint32_t* __restrict__ cursor, const uint8_t* __restrict__ dup,
                                   uint64_t* __restrict__ codes, uint32_t* __restrict__ index) {
  for (int64_t j = (int64_t)blockIdx.x * WG + threadIdx.x; j < nw; j += (int64_t)gridDim.x * WG) {
    const uint64_t w = wl[j];
    const uint32_t pos = atomicAdd(&cursor[part_bucket(w, part)], 1u);
    codes[pos] = w;
    index[pos] = (uint32_t)j | (dup[j] ? 0x80000000u : 0u);
  }
}

// occupied buckets of a provisional table (~ the distinct block values)
__global__ void count_nonzero_kernel(const uint32_t* __restrict__ counts, int64_t nbuckets,
                                     unsigned long long* __restrict__ out) {
  uint32_t c = 0;
  for (int64_t b = (int64_t)blockIdx.x * WG + threadIdx.x; b < nbuckets; b += (int64_t)gridDim.x * WG)
    c += counts[b] != 0;
  for (int o = 32; o; o >>= 1) c += __shfl_xor(c, o);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(out, (unsigned long long)c);
}

// Duplicate whitelist codes (the same code at two indices always ties): the codes sorted
// with their indices, equal neighbours flag both indices.  No per-bucket pair scan, so a
// block value shared by many codes costs nothing extra.
__global__ void flag_dups_kernel(const uint64_t* __restrict__ sorted, const uint32_t* __restrict__ idx, int64_t nw,
                                 uint8_t* __restrict__ dup) {
  for (int64_t k = (int64_t)blockIdx.x * WG + threadIdx.x; k < nw; k += (int64_t)gridDim.x * WG) {
    const uint64_t c = sorted[k];
    const bool d = (k > 0 && sorted[k - 1] == c) || (k + 1 < nw && sorted[k + 1] == c);
    dup[idx[k]] = d ? 1 : 0;
  }
}

__global__ void iota_kernel(uint32_t* __restrict__ v, int64_t n) {
  for (int64_t k = (int64_t)blockIdx.x * WG + threadIdx.x; k < n; k += (int64_t)gridDim.x * WG) v[k] = (uint32_t)k;
}

// Per-probe tables, passed by value (kernarg -> SGPRs) so every load is a global load.
struct Tables {
  Part part[MAX_PARTS];
  const uint32_t* off[MAX_PARTS];  // bucket b's entries are [off[b], off[b + 1])
  const uint64_t* code[MAX_PARTS];
  const uint32_t* index[MAX_PARTS];
};

template <int KIND, int NP>
__global__ __launch_bounds__(WG) void nearest_query_kernel(const uint64_t* __restrict__ queries,
                                                           int64_t nq, Tables tb, int max_d,
                                                           int32_t* __restrict__ out_index,
                                                           uint8_t* __restrict__ out_dist) {
  const int64_t i = (int64_t)blockIdx.x * WG + threadIdx.x;
  if (i >= nq) return;
  const uint64_t q = queries[i];
  uint2 r[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) {  // all in flight
    const uint32_t* o = tb.off[p] + part_bucket(q, tb.part[p]);
    r[p] = make_uint2(o[0], o[1]);
  }
  int best_d = max_d + 1, best_j = -1;
  bool tie = false, exact_unique = false;
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    // an exact hit on a code that occurs once cannot tie (every other code is >= 1 away):
    // the remaining probes' entry reads are skipped
    if (exact_unique) break;
    for (uint32_t t = r[p].x; t < r[p].y; ++t) {
      const uint64_t w = tb.code[p][t];
      const int d = KIND == 2 ? dist2(q, w) : dist3(q, w);
      if (d <= best_d && d <= max_d) {  // rare: only candidates within max_d read their index
        const uint32_t jf = tb.index[p][t];
        const int j = (int)(jf & 0x7FFFFFFFu);
        if (d < best_d) {
          best_d = d;
          best_j = j;
          tie = false;
          exact_unique = d == 0 && !(jf >> 31);
        } else if (j != best_j) {
          tie = true;
        }
      }
    }
  }
  out_index[i] = best_j < 0 ? -1 : (tie ? -2 : best_j);
  out_dist[i] = best_j < 0 ? (uint8_t)255 : (uint8_t)best_d;
}

// ---------------------------------------------------------------- open-addressing multi-index
// When the whitelist's keys are (nearly) unique -- max_d = 0 (key = the whole code), or
// max_d = 1..2 with P = max_d + 2 blocks and keys = PAIRS of blocks (a code within max_d
// agrees exactly on >= 2 of the P blocks, so on at least one pair): config 4 has three
// 10-11-base pair keys for 737K codes -- every key gets a hash table of 16-byte slots
// {code, index} in 64-byte groups of 4 (linear probing from the key's group, load <= 1/2).
// A query reads one group per table, all tables' groups in flight at once: one dependent
// round trip per query instead of an offset load followed by a scan of ~11 entries per
// probe; a group without a free slot continues in the next (rare).
constexpr uint32_t kEmpty = 0xFFFFFFFFu;
constexpr int kGroup = 4;  // slots per group (64 B)
constexpr int MAX_KEYS = 6;  // C(4, 2): max_d = 2

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

struct OTable {
  uint64_t keymask;  // OR of the key's block masks
  uint64_t gmask;    // groups - 1
  uint4* slots;      // {code lo, code hi, index | kEmpty, 1 if the code occurs twice}
};
struct OTables {
  OTable t[MAX_KEYS];
};

__global__ void oa_clear_kernel(uint4* __restrict__ slots, int64_t nslots) {
  for (int64_t k = (int64_t)blockIdx.x * WG + threadIdx.x; k < nslots; k += (int64_t)gridDim.x * WG)
    slots[k] = make_uint4(0u, 0u, kEmpty, 0u);
}

__global__ void oa_insert_kernel(const uint64_t* __restrict__ wl, int64_t nw, const uint8_t* __restrict__ dup,
                                 OTable tb) {
  const int64_t nslots = (int64_t)(tb.gmask + 1) * kGroup;
  for (int64_t j = (int64_t)blockIdx.x * WG + threadIdx.x; j < nw; j += (int64_t)gridDim.x * WG) {
    const uint64_t w = wl[j];
    int64_t sidx = (int64_t)(mix64(w & tb.keymask) & tb.gmask) * kGroup;
    for (int64_t step = 0; step < nslots; ++step, sidx = (sidx + 1) & (nslots - 1)) {
      uint32_t* ix = reinterpret_cast<uint32_t*>(tb.slots + sidx) + 2;
      if (atomicCAS(ix, kEmpty, (uint32_t)j) == kEmpty) {
        uint32_t* c = reinterpret_cast<uint32_t*>(tb.slots + sidx);
        c[0] = (uint32_t)w;
        c[1] = (uint32_t)(w >> 32);
        c[3] = dup[j];
        break;
      }
    }
  }
}

template <int KIND, int T>
__global__ __launch_bounds__(WG) void oa_query_kernel(const uint64_t* __restrict__ queries, int64_t nq, OTables tb,
                                                      int max_d, int32_t* __restrict__ out_index,
                                                      uint8_t* __restrict__ out_dist) {
  const int64_t i = (int64_t)blockIdx.x * WG + threadIdx.x;
  if (i >= nq) return;
  const uint64_t q = queries[i];
  int best_d = max_d + 1, best_j = -1;
  bool tie = false;
  uint64_t grp[T];
  uint4 v[T][kGroup];
  auto load_group = [&](int t) {
    grp[t] = mix64(q & tb.t[t].keymask) & tb.t[t].gmask;
    const uint4* g = tb.t[t].slots + grp[t] * kGroup;
#pragma unroll
    for (int k = 0; k < kGroup; ++k) v[t][k] = g[k];
  };
  // Table 0 first: an exact hit on a code that occurs once is the answer (every other code
  // is >= 1 away) and the other tables are never read -- half of config 4's queries.  Any
  // exact match shares every key, so it is always in table 0's probe sequence.
  load_group(0);
  bool exact_unique = false;
#pragma unroll
  for (int k = 0; k < kGroup; ++k) {
    const uint4 e = v[0][k];
    if (e.z != kEmpty && ((uint64_t)e.y << 32 | e.x) == q && !e.w) {
      exact_unique = true;
      best_d = 0;
      best_j = (int)e.z;
    }
  }
  if (exact_unique) {
    out_index[i] = best_j;
    out_dist[i] = 0;
    return;
  }
#pragma unroll
  for (int t = 1; t < T; ++t) load_group(t);  // the other tables' groups in flight together
  auto visit = [&](const uint4 e) {
    const uint64_t w = ((uint64_t)e.y << 32) | e.x;
    const int d = KIND == 2 ? dist2(q, w) : dist3(q, w);
    if (d <= best_d && d <= max_d) {
      const int j = (int)e.z;
      if (d < best_d) {
        best_d = d;
        best_j = j;
        tie = false;
      } else if (j != best_j) {
        tie = true;
      }
    }
  };
#pragma unroll
  for (int t = 0; t < T; ++t) {
    bool open = false;  // a free slot ends the key's probe sequence
#pragma unroll
    for (int k = 0; k < kGroup; ++k) {
      if (v[t][k].z == kEmpty) open = true;
      else if (!open) visit(v[t][k]);
    }
    for (uint64_t g = grp[t]; !open;) {  // the group was full: the next one (rare)
      g = (g + 1) & tb.t[t].gmask;
      const uint4* gp = tb.t[t].slots + g * kGroup;
      for (int k = 0; k < kGroup && !open; ++k) {
        const uint4 e = gp[k];
        if (e.z == kEmpty) open = true;
        else visit(e);
      }
    }
  }
  out_index[i] = best_j < 0 ? -1 : (tie ? -2 : best_j);
  out_dist[i] = best_j < 0 ? (uint8_t)255 : (uint8_t)best_d;
}

// ---------------------------------------------------------------- half-key tables (max_d <= 1)
// For max_d <= 1 and a whitelist whose G in-code positions are all A/C/G/T (every TwoBit
// code; ThreeBit codes whose triplets are 1..4), split the positions into a high half A =
// [GB, G) and a low half B = [0, GB) and give every half a 2-bit digit key (<= 8 digits:
// 16 bits).  A code within distance 1 of the query agrees with it exactly on A or on B.
// Two tables of the whitelist: sorted by (A, B) -- offA[key] .. offA[key + 1] holds the B
// keys of the codes whose A key is `key`, as uint16 -- and sorted by (B, A) with the A keys.
// At 737K 16-base codes both tables with their offsets take 3.5 MB: every XCD's 4 MB L2
// holds them, so a query costs L2 hits instead of Infinity-Cache line fetches (the open-
// addressing tables' 96 MB did not fit anywhere closer).  A query scans its A bucket (~11
// entries, 16 B = 8 entries per load); an exact hit there settles it (every exact match lies
// in that bucket, and the other table only adds codes >= 1 away); otherwise its B bucket,
// skipping the codes that agree on A too (those were in the A bucket).  Each whitelist
// entry is visited at most once, so two candidates at the best distance are two indices: a
// tie.  The kernel writes the winner's table position (A order: p, B order: nw + p); a second
// pass maps it to the whitelist index through permAB, packed to ceil(log2 nw) bits per entry.
// Entries are tested two per dword (SWAR): per 16-bit field the mismatching digits
// m = ((x | x >> 1) & 0x5555) | invalid, x = entry ^ key; then d >= 1 iff m != 0 and d >= 2
// iff m with its lowest set bit cleared != 0, both read off bit 15 of field + 0x7FFF (no
// field exceeds 0x5555, so no carry leaves a field).
// Query groups above the table's G positions are compared with the whitelist's zeros: they
// add the same E to every distance.  A query digit that is not A/C/G/T (N, 0, 5, 7 in
// ThreeBit) matches no whitelist digit.
struct Halves {
  int G, GA, GB;            // positions; high half A = [GB, G) (GA digits), low half B = [0, GB)
  const uint32_t* offA;     // [4^GA + 1]
  const uint16_t* entA;     // [nw] B keys, codes sorted by (A, B)
  const uint32_t* offB;     // [4^GB + 1]
  const uint16_t* entB;     // [nw] A keys, codes sorted by (B, A)
  const uint32_t* permAB;   // [2 nw] whitelist index of each A-order, then B-order position (build only;
                            // the index pass reads it packed, sct_nearest_plan::perm_packed)
  int64_t nw;
  // Digit keys: any order of A/C/G/T answers the same (a key only has to be equal or not), so the
  // plan takes the order the whitelist is sorted in, if any -- alphabetical (a 10x whitelist file),
  // TwoBit's A C T G (numerically sorted TwoBit codes) or ThreeBit's C A G T -- as
  // d1 = the base's TwoBit high bit, d0 = (TwoBit low bit) ^ dinv ^ (dalpha & d1).  In key order
  // A-order position p is whitelist index p: the query kernel then writes whitelist indices itself,
  // reading the packed permutation only for a winner found through the B table, and the index
  // pass is skipped (ident_a).
  uint32_t dinv, dalpha;  // 0 or ~0u
  int ident_a;
  // ident_a: rankB[p] = the rank of B-order entry p's code inside its A bucket (< 256; null when a
  // bucket holds more), so a B-table winner's whitelist index is offA[its A key] + rankB[p]: a
  // 0.74 MB byte array beside the hot offsets instead of the 1.85 MB half of the permutation
  const uint8_t* rankB;
  const uint32_t* perm_packed;
  int pbits;
};

// Stride-3 -> stride-2 compaction of the 8 fields of a 24-bit ThreeBit half (field p at bit
// 3p moves to bit 2p): three shift stages, stage j moving the fields whose p has bit j set.
template <int W>
constexpr uint32_t compact_mask(int j) {
  uint32_t m = 0;
  for (int p = 0; p < 8; ++p)
    if ((p >> j) & 1) m |= ((1u << W) - 1) << (3 * p - (p & ((1 << j) - 1)));
  return m;
}
template <int W>
__device__ __forceinline__ uint32_t compact3to2(uint32_t x) {
  x = (x & ~compact_mask<W>(0)) | ((x & compact_mask<W>(0)) >> 1);
  x = (x & ~compact_mask<W>(1)) | ((x & compact_mask<W>(1)) >> 2);
  x = (x & ~compact_mask<W>(2)) | ((x & compact_mask<W>(2)) >> 4);
  return x;
}

// one ThreeBit half of `nd` triplets (bits 0..3 nd - 1 of h) -> 2-bit digit key in the plan's
// digit order (Halves::dinv / dalpha) and the invalid digits spread to the key's even bits
__device__ __forceinline__ void half3(uint32_t h, int nd, uint32_t dinv, uint32_t dalpha, uint32_t& key,
                                      uint32_t& spread) {
  constexpr uint32_t M = 0x249249u;  // bit 3p, p < 8
  const uint32_t live = nd >= 8 ? M : (M & ((1u << (3 * nd)) - 1));
  const uint32_t a = h & live, b = (h >> 1) & live, c = (h >> 2) & live;
  // valid triplets C 1, A 2, G 3, T 4 (abc = 100, 010, 110, 001): d1 = (a & b) | c (G, T), and a
  // is TwoBit's low bit (C, G); d0 = a ^ dinv ^ (dalpha & d1)
  const uint32_t valid = (~c & (a | b)) | (c & ~a & ~b);
  const uint32_t d1 = (a & b) | c;
  const uint32_t dig = ((a ^ dinv ^ (dalpha & d1)) & live) | (d1 << 1);
  key = compact3to2<2>(dig);
  spread = compact3to2<1>(live & ~valid);
}

template <int KIND>
__device__ __forceinline__ void halves_of(uint64_t q, const Halves& h, uint32_t& kA, uint32_t& sA, uint32_t& kB,
                                          uint32_t& sB, int& E) {
  const int top = KIND * h.G;
  const uint64_t hi = top >= 64 ? 0ull : q >> top;
  if constexpr (KIND == 2) {
    E = __popcll((hi | (hi >> 1)) & 0x5555555555555555ull);
    // TwoBit digits A 0, C 1, T 2, G 3: d0 ^= dinv ^ (dalpha & d1)
    const uint32_t x = (uint32_t)(q & 0xFFFFFFFFull), f = (h.dinv & 0x55555555u) ^ (h.dalpha & (x >> 1) & 0x55555555u);
    kB = (x ^ f) & ((1u << (2 * h.GB)) - 1);
    kA = ((x ^ f) >> (2 * h.GB)) & ((1u << (2 * h.GA)) - 1);
    sA = sB = 0;
  } else {
    E = __popcll((hi | (hi >> 1) | (hi >> 2)) & 0x9249249249249249ull);
    half3((uint32_t)(q & ((1u << (3 * h.GB)) - 1)), h.GB, h.dinv, h.dalpha, kB, sB);
    half3((uint32_t)((q >> (3 * h.GB)) & ((1u << (3 * h.GA)) - 1)), h.GA, h.dinv, h.dalpha, kA, sA);
  }
}

typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
// Entries [b, e) of a uint16 table against the half key k (invalid digits `sp` spread to the
// even bits): z0 / z1 count the entries at half distance 0 / 1, p0 / p1 the position of one.
template <bool LEVEL0>
__device__ __forceinline__ void scan_chunk(const uint4 v, uint32_t c, uint32_t b, uint32_t e, uint32_t k2, uint32_t sp2,
                                           int& n0, uint32_t& p0, int& n1, uint32_t& p1, uint32_t& v1) {
  // in-range entries of the chunk, in the layout below: entry 2k at bit 2k, 2k + 1 at 16 + 2k
  const uint32_t lo = b > c ? b - c : 0u, hi = e - c < 8u ? e - c : 8u;
  const uint32_t in8 = ((1u << hi) - 1u) & ~((1u << lo) - 1u);
  const uint32_t inr = (in8 & 0x55u) | ((in8 & 0xAAu) << 15);
  uint32_t f0 = 0, f1 = 0;
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t x = (w[q] ^ k2) | sp2;  // an invalid query digit differs from every entry digit
    const uint32_t m = (x | (x >> 1)) & 0x55555555u;
    const u16x2 mh = __builtin_bit_cast(u16x2, m);
    const uint32_t t = m & __builtin_bit_cast(uint32_t, (u16x2)(mh - (u16x2){1, 1}));  // per half: m & (m - 1)
    const uint32_t ge1 = (m + 0x7FFF7FFFu) & 0x80008000u, ge2 = (t + 0x7FFF7FFFu) & 0x80008000u;
    if constexpr (LEVEL0) f0 |= ((~ge1 & 0x80008000u) >> 15) << (2 * q);
    f1 |= ((ge1 & ~ge2) >> 15) << (2 * q);
  }
  if constexpr (LEVEL0) {
    f0 &= inr;
    if (f0) {
      n0 += __popc(f0);
      const uint32_t bit = __ffs(f0) - 1;
      p0 = c + (bit < 16 ? bit : bit - 15);
    }
  }
  f1 &= inr;
  if (f1) {
    n1 += __popc(f1);
    const uint32_t bit = __ffs(f1) - 1;
    p1 = c + (bit < 16 ? bit : bit - 15);
    const uint32_t q = (bit & 15) >> 1, d = q == 0 ? v.x : q == 1 ? v.y : q == 2 ? v.z : v.w;
    v1 = (d >> (bit & 16)) & 0xFFFFu;  // the entry's key (the other half of its code)
  }
}

// Entries [b, e) of a uint16 table against the half key k (invalid digits `sp` spread to the
// even bits): z0 / z1 count the entries at half distance 0 / 1, p0 / p1 the position of one.
// Chunks of 8 entries go three at a time: all three 16-B loads (the ones inside [b, e)) are
// issued before any is tested, so the later ones (usually in the same line) ride on the first's
// miss instead of making their own dependent L2 requests (one, two, three, four at a time:
// 2.46 / 2.23 / 2.17 / 2.19 ms per 100M queries, profiles/ab_nearest_chunks_r03.jsonl).  The
// first chunk starts at b's dword, not its 16-B chunk: a wave runs as many chunks as its fullest
// lane spans, and the 16-B rounding added one on most waves (1.5-2 %, ab_nearest_align_r06.json).
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
template <bool LEVEL0, int kGroup = 3>
__device__ __forceinline__ void scan_half(const uint16_t* __restrict__ ent, uint32_t b, uint32_t e, uint32_t k,
                                          uint32_t sp, int& n0, uint32_t& p0, int& n1, uint32_t& p1, uint32_t& v1) {
  const uint32_t k2 = k | (k << 16), sp2 = sp | (sp << 16);
  for (uint32_t c = b & ~1u; c < e; c += 8 * kGroup) {
    uint4 v[kGroup];
#pragma unroll
    for (int j = 0; j < kGroup; ++j) {
      v[j] = make_uint4(0, 0, 0, 0);
      if (j == 0 || c + 8 * j < e) {
        const u32x4_a4 x = *reinterpret_cast<const u32x4_a4*>(ent + c + 8 * j);
        v[j] = make_uint4(x.x, x.y, x.z, x.w);
      }
    }
#pragma unroll
    for (int j = 0; j < kGroup; ++j)
      if (j == 0 || c + 8 * j < e) scan_chunk<LEVEL0>(v[j], c + 8 * j, b, e, k2, sp2, n0, p0, n1, p1, v1);
  }
}

typedef uint32_t u32x2_a4 __attribute__((ext_vector_type(2), aligned(4)));
__device__ __forceinline__ int32_t unpack_perm(const uint32_t* __restrict__ packed, int pbits, int32_t p) {
  const uint64_t bo = (uint64_t)p * pbits;
  const u32x2_a4 d = *reinterpret_cast<const u32x2_a4*>(packed + (bo >> 5));  // one 8-byte load
  return (int32_t)(((((uint64_t)d.y << 32) | d.x) >> (bo & 31)) & ((1ull << pbits) - 1));
}

// IDX (Halves::ident_a): out_pos receives whitelist indices (a B-table winner's through the packed
// permutation, read here), else table positions for halves_index_kernel
template <int KIND, bool IDX>
__global__ __launch_bounds__(WG) void halves_query_kernel(const uint64_t* __restrict__ queries, int64_t nq, Halves h,
                                                          int max_d, int32_t* __restrict__ out_pos,
                                                          uint8_t* __restrict__ out_dist) {
  const int64_t i = (int64_t)blockIdx.x * WG + threadIdx.x;
  if (i >= nq) return;
  const uint64_t q = __builtin_nontemporal_load(queries + i);
  uint32_t kA, sA, kB, sB;
  int E;
  halves_of<KIND>(q, h, kA, sA, kB, sB, E);
  const int eff = max_d - E;  // in-table distance allowed
  int nA0 = 0, nA1 = 0, nB0 = 0, nB1 = 0;
  uint32_t pA0 = 0, pA1 = 0, pB0 = 0, pB1 = 0, vA1 = 0, vB1 = 0;
  if (eff >= 0 && sA == 0)  // the A bucket: codes agreeing with q on A
    scan_half<true>(h.entA, h.offA[kA], h.offA[kA + 1], kB, sB, nA0, pA0, nA1, pA1, vA1);
  // an exact hit (unique or not) is final: the B table holds no other code at distance 0;
  // in the B bucket the codes at A distance 0 are the A bucket's exact hits, not counted
  if (eff >= 1 && nA0 == 0 && sB == 0)
    scan_half<false>(h.entB, h.offB[kB], h.offB[kB + 1], kA, sA, nB0, pB0, nB1, pB1, vB1);
  int32_t pos = -1;
  uint8_t dist = 255;
  if (nA0) {
    pos = nA0 == 1 ? (int32_t)pA0 : -2;
    dist = (uint8_t)E;
  } else if (eff >= 1 && nA1 + nB1) {
    if (nA1 + nB1 >= 2) pos = -2;
    else if (nA1) pos = (int32_t)pA1;
    else if (!IDX) pos = (int32_t)(h.nw + pB1);
    else if (h.rankB) pos = (int32_t)(h.offA[vB1] + h.rankB[pB1]);  // both loads at once
    else pos = unpack_perm(h.perm_packed, h.pbits, (int32_t)(h.nw + pB1));
    dist = (uint8_t)(1 + E);
  }
  __builtin_nontemporal_store(pos, out_pos + i);
  __builtin_nontemporal_store(dist, out_dist + i);
}

// permAB packed to pbits per entry (the whitelist index needs ceil(log2 nw) bits: 20 at 737K,
// 3.7 MB instead of 5.9 -- it fits an XCD's 4 MB L2 while the index pass runs): output dword w
// gathers the bits of the (at most three) entries overlapping bits [32 w, 32 w + 32)
__global__ void pack_perm_kernel(const uint32_t* __restrict__ perm, int64_t n, int pbits, int64_t ndw,
                                 uint32_t* __restrict__ out) {
  for (int64_t w = (int64_t)blockIdx.x * WG + threadIdx.x; w < ndw; w += (int64_t)gridDim.x * WG) {
    uint32_t v = 0;
    for (int64_t e = (32 * w) / pbits; e < n && e * pbits < 32 * w + 32; ++e) {
      const int64_t sh = e * pbits - 32 * w;
      v |= sh >= 0 ? perm[e] << sh : perm[e] >> (-sh);
    }
    out[w] = v;
  }
}

// table positions -> whitelist indices (-1 / -2 pass through): four queries per lane per step,
// their packed-perm loads independent
__global__ __launch_bounds__(WG) void halves_index_kernel(int32_t* __restrict__ idx, int64_t nq,
                                                          const uint32_t* __restrict__ packed, int pbits, bool vec) {
  typedef int v4i __attribute__((ext_vector_type(4)));
  const int64_t n4 = vec ? nq / 4 : 0;  // vec: idx is 16-B aligned
  v4i* idx4 = reinterpret_cast<v4i*>(idx);
  for (int64_t i = (int64_t)blockIdx.x * WG + threadIdx.x; i < n4; i += (int64_t)gridDim.x * WG) {
    v4i p = __builtin_nontemporal_load(idx4 + i);
    v4i o;
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = p[k] >= 0 ? unpack_perm(packed, pbits, p[k]) : p[k];
    __builtin_nontemporal_store(o, idx4 + i);
  }
  for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * WG + threadIdx.x; i < nq; i += (int64_t)gridDim.x * WG)
    if (idx[i] >= 0) idx[i] = unpack_perm(packed, pbits, idx[i]);
}

// Half-key table build (round 4: a counting sort by bucket with no host synchronisation before
// the end -- the order inside a bucket is irrelevant, a query scans its whole bucket):
//   count    per code its A and B keys: atomic bucket counts; *bad = 1 if a code has a digit that
//            is not A/C/G/T in its G positions or any bit above them (the layout is then dropped)
//   scan     one workgroup: offsets of both tables, the cursors in place
//   scatter  per code: one slot in its A bucket (entry = its B key) and one in its B bucket
//            (entry = its A key), the whitelist index of both slots into permAB
// the digit order halves_pick_order_kernel chose (device words: dinv, dalpha, ident_a)
__device__ __forceinline__ void take_order(Halves& h, const unsigned* __restrict__ order) {
  h.dinv = order[0];
  h.dalpha = order[1];
  h.ident_a = (int)order[2];
}

template <int KIND>
__global__ void halves_count_kernel(const uint64_t* __restrict__ wl, int64_t nw, Halves h,
                                    uint32_t* __restrict__ cntA, uint32_t* __restrict__ cntB,
                                    unsigned* __restrict__ bad, const unsigned* __restrict__ order) {
  take_order(h, order);
  bool b = false;
  for (int64_t j = (int64_t)blockIdx.x * WG + threadIdx.x; j < nw; j += (int64_t)gridDim.x * WG) {
    uint32_t kA, sA, kB, sB;
    int E;
    halves_of<KIND>(wl[j], h, kA, sA, kB, sB, E);
    b |= (E | sA | sB) != 0;
    atomicAdd(&cntA[kA], 1u);
    atomicAdd(&cntB[kB], 1u);
  }
  if (b) atomicOr(bad, 1u);
}

// exclusive scan of cnt[0, n) by one 1024-thread workgroup into off[0, n] and cnt (the cursors);
// n = 4096 k (k <= 16: half keys of 6-8 digits) as 16-B vectors, all of a thread's loads in
// flight at once (one element at a time the scan of 2 x 65,536 counts took 0.28 ms)
__device__ __forceinline__ void block_scan_offsets(uint32_t* __restrict__ cnt, int64_t n, uint32_t* __restrict__ off,
                                                   uint32_t* wsum) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  if (n % 4096 == 0 && n <= 65536) {
    const int per4 = (int)(n / 4096);  // 16-B vectors per thread
    uint4* c4 = reinterpret_cast<uint4*>(cnt) + (int64_t)t * per4;
    uint4* o4 = reinterpret_cast<uint4*>(off) + (int64_t)t * per4;
    uint4 v[16];
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (k < per4) v[k] = c4[k];
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (k < per4) s += v[k].x + v[k].y + v[k].z + v[k].w;
    uint32_t is = s;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t a = __shfl_up(is, d);
      if (lane >= d) is += a;
    }
    if (lane == 63) wsum[wave] = is;
    __syncthreads();
    uint32_t run = is - s;
    for (int w = 0; w < wave; ++w) run += wsum[w];
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (k < per4) {
        uint4 r;
        r.x = run;
        r.y = r.x + v[k].x;
        r.z = r.y + v[k].y;
        r.w = r.z + v[k].z;
        run = r.w + v[k].w;
        o4[k] = r;
        c4[k] = r;
      }
    if (t == 1023) off[n] = run;
    __syncthreads();  // wsum is reused
    return;
  }
  const int64_t per = (n + 1023) / 1024, b = std::min<int64_t>(n, t * per), e = std::min<int64_t>(n, b + per);
  uint32_t s = 0;
  for (int64_t i = b; i < e; ++i) s += cnt[i];
  uint32_t is = s;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t a = __shfl_up(is, d);
    if (lane >= d) is += a;
  }
  if (lane == 63) wsum[wave] = is;
  __syncthreads();
  uint32_t run = is - s;
  for (int w = 0; w < wave; ++w) run += wsum[w];
  for (int64_t i = b; i < e; ++i) {
    const uint32_t c = cnt[i];
    off[i] = run;
    cnt[i] = run;
    run += c;
  }
  if (t == 1023) off[n] = run;
  __syncthreads();  // wsum is reused
}

__global__ __launch_bounds__(1024) void halves_scan_kernel(uint32_t* __restrict__ cntA, int64_t nA,
                                                           uint32_t* __restrict__ offA, uint32_t* __restrict__ cntB,
                                                           int64_t nB, uint32_t* __restrict__ offB) {
  __shared__ uint32_t wsum[16];
  block_scan_offsets(cntA, nA, offA, wsum);
  block_scan_offsets(cntB, nB, offB, wsum);
}

// The candidate digit orders (Halves::dinv, dalpha) and whether the whitelist is out of (A, B) key
// order under each: unsorted[o] = 1 if some code's key exceeds the next one's
constexpr int kOrders = 3;
constexpr uint32_t kOrderInv[kOrders] = {0u, 0u, ~0u}, kOrderAlpha[kOrders] = {~0u, 0u, 0u};  // ACGT, ACTG, CAGT
template <int KIND>
__global__ void halves_order_kernel(const uint64_t* __restrict__ wl, int64_t nw, Halves h,
                                    unsigned* __restrict__ unsorted) {
  bool u[kOrders] = {};
  for (int64_t j = (int64_t)blockIdx.x * WG + threadIdx.x; j + 1 < nw; j += (int64_t)gridDim.x * WG) {
    const uint64_t w0 = wl[j], w1 = wl[j + 1];
#pragma unroll
    for (int o = 0; o < kOrders; ++o) {
      h.dinv = kOrderInv[o];
      h.dalpha = kOrderAlpha[o];
      uint32_t kA, sA, kB, sB, kA1, kB1;
      int E;
      halves_of<KIND>(w0, h, kA, sA, kB, sB, E);
      halves_of<KIND>(w1, h, kA1, sA, kB1, sB, E);
      u[o] |= kA > kA1 || (kA == kA1 && kB > kB1);
    }
  }
  // one atomic per wave, and none once the flag is set (every wave of an unsorted whitelist finds
  // a pair out of order: 11K atomics on three words serialised at L2 cost 0.3 ms)
#pragma unroll
  for (int o = 0; o < kOrders; ++o)
    if (__ballot(u[o]) && (threadIdx.x & 63) == 0 && !__hip_atomic_load(unsorted + o, __ATOMIC_RELAXED,
                                                                        __HIP_MEMORY_SCOPE_AGENT))
      atomicOr(unsorted + o, 1u);
}

// order[0..2] = dinv, dalpha, ident_a of the first candidate order the whitelist is sorted in, or
// alphabetical keys with ident_a = 0 (the index pass then maps the A-table positions)
__global__ void halves_pick_order_kernel(const unsigned* __restrict__ unsorted, unsigned* __restrict__ order) {
  int o = 0;
  while (o < kOrders && unsorted[o]) ++o;
  order[0] = kOrderInv[o < kOrders ? o : 0];
  order[1] = kOrderAlpha[o < kOrders ? o : 0];
  order[2] = o < kOrders ? 1u : 0u;
}

template <int KIND>
__global__ void halves_scatter_kernel(const uint64_t* __restrict__ wl, int64_t nw, Halves h,
                                      uint32_t* __restrict__ curA, uint32_t* __restrict__ curB,
                                      uint16_t* __restrict__ entA, uint16_t* __restrict__ entB,
                                      uint32_t* __restrict__ perm, const unsigned* __restrict__ order,
                                      uint8_t* __restrict__ rankB, unsigned* __restrict__ rank_over) {
  take_order(h, order);
  const bool sorted = h.ident_a != 0;  // in key order: code j's A-table slot is j
  bool over = false;
  for (int64_t j = (int64_t)blockIdx.x * WG + threadIdx.x; j < nw; j += (int64_t)gridDim.x * WG) {
    uint32_t kA, sA, kB, sB;
    int E;
    halves_of<KIND>(wl[j], h, kA, sA, kB, sB, E);
    const uint32_t pA = sorted ? (uint32_t)j : atomicAdd(&curA[kA], 1u), pB = atomicAdd(&curB[kB], 1u);
    entA[pA] = (uint16_t)kB;
    perm[pA] = (uint32_t)j;
    entB[pB] = (uint16_t)kA;
    perm[nw + pB] = (uint32_t)j;
    if (sorted) {
      const uint32_t r = pA - h.offA[kA];  // the code's rank inside its A bucket
      over |= r > 255u;
      rankB[pB] = (uint8_t)r;
    }
  }
  if (over) atomicOr(rank_over, 1u);
}

template <int KIND>
void launch_oa_query(int nt, unsigned blocks, hipStream_t s, const uint64_t* q, int64_t nq, const OTables& tb,
                     int max_d, int32_t* idx, uint8_t* dist) {
#define SCT_OQ(T)                                                                                       \
  case T:                                                                                               \
    hipLaunchKernelGGL((oa_query_kernel<KIND, T>), dim3(blocks), dim3(WG), 0, s, q, nq, tb, max_d, idx, \
                       dist);                                                                           \
    break;
  switch (nt) {
    SCT_OQ(1) SCT_OQ(3) SCT_OQ(6)
    default: break;
  }
#undef SCT_OQ
}

template <int KIND>
void launch_query(int np, unsigned blocks, hipStream_t s, const uint64_t* q, int64_t nq,
                  const Tables& tb, int max_d, int32_t* idx, uint8_t* dist) {
#define SCT_NQ(NP)                                                                                 \
  case NP:                                                                                         \
    hipLaunchKernelGGL((nearest_query_kernel<KIND, NP>), dim3(blocks), dim3(WG), 0, s, q, nq, tb, \
                       max_d, idx, dist);                                                          \
    break;
  switch (np) {
    SCT_NQ(1) SCT_NQ(2) SCT_NQ(3) SCT_NQ(4) SCT_NQ(5) SCT_NQ(6) SCT_NQ(7) SCT_NQ(8)
    default: break;
  }
#undef SCT_NQ
}

unsigned grid_for(int64_t n, int64_t cap = 16384) {
  const int64_t b = sct::ceil_div(n, WG);
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(b, cap));
}

}  // namespace

// dup[j] = 1 if whitelist code j occurs more than once (sorted (code, index), equal
// neighbours); a device buffer of nw bytes, ready on `s` when this returns.
static int compute_dups(const uint64_t* d_whitelist, int64_t nw, uint8_t* dup, hipStream_t s) {
  SCT_HIP(hipMemsetAsync(dup, 0, (size_t)std::max<int64_t>(nw, 1), s));
  if (nw < 2) return SCT_OK;
  size_t sort_bytes = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                           (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)nw, 0, 64, s);
  sct::DevBuf tmp, skeys, sidx, iota;
  SCT_HIP(tmp.alloc(sort_bytes));
  SCT_HIP(skeys.alloc((size_t)nw * 8));
  SCT_HIP(sidx.alloc((size_t)nw * 4));
  SCT_HIP(iota.alloc((size_t)nw * 4));
  hipLaunchKernelGGL(iota_kernel, dim3(grid_for(nw, 4096)), dim3(WG), 0, s, (uint32_t*)iota.p, nw);
  SCT_HIP(hipcub::DeviceRadixSort::SortPairs(tmp.p, sort_bytes, d_whitelist, (uint64_t*)skeys.p,
                                             (const uint32_t*)iota.p, (uint32_t*)sidx.p, (int)nw, 0, 64, s));
  hipLaunchKernelGGL(flag_dups_kernel, dim3(grid_for(nw, 4096)), dim3(WG), 0, s, (const uint64_t*)skeys.p,
                     (const uint32_t*)sidx.p, nw, dup);
  SCT_LAUNCH_CHECK();
  SCT_HIP(hipStreamSynchronize(s));  // the scratch dies here
  return SCT_OK;
}

struct sct_nearest_plan {
  int kind = 2, max_d = 0, nparts = 0, code_bits = 0;
  int64_t nw = 0;
  bool halves = false;  // half-key tables (Halves) for max_d <= 1
  Halves hv{};
  void* hv_mem[1] = {};  // one block: offA, offB, entA, entB, packed permAB
  uint32_t* perm_packed = nullptr;  // permAB at pbits per entry (+ 2 dwords of padding), inside hv_mem[0]
  int pbits = 0;
  int nkeys = 0;  // > 0: open-addressing multi-index (OTables); 0: CSR per block (Parts)
  OTables ot{};
  Parts parts{};
  int64_t nbuckets[MAX_PARTS] = {};
  uint32_t* d_off[MAX_PARTS] = {};
  uint64_t* d_code[MAX_PARTS] = {};
  uint32_t* d_index[MAX_PARTS] = {};
  // recorded after every query on its stream: destroy waits on it, so freeing the tables never
  // races a query still in flight (a caller may destroy right after enqueueing one)
  hipEvent_t last_query = nullptr;
};

extern "C" int sct_nearest_plan_destroy(sct_nearest_plan* p) {
  if (!p) return SCT_OK;
  if (p->last_query) {
    (void)hipEventSynchronize(p->last_query);
    (void)hipEventDestroy(p->last_query);
  }
  for (void* m : p->hv_mem)
    if (m) (void)hipFree(m);
  for (int k = 0; k < MAX_KEYS; ++k)
    if (p->ot.t[k].slots) (void)hipFree(p->ot.t[k].slots);
  for (int k = 0; k < MAX_PARTS; ++k) {
    if (p->d_off[k]) (void)hipFree(p->d_off[k]);
    if (p->d_code[k]) (void)hipFree(p->d_code[k]);
    if (p->d_index[k]) (void)hipFree(p->d_index[k]);
  }
  delete p;
  return SCT_OK;
}

// The half-key tables, if the whitelist allows them (SCT_OK with p->halves set), else SCT_OK
// with p->halves false (the caller takes another layout).  One device allocation for the
// plan's tables, scratch from the library's pool, one synchronisation (for the layout check).
static int build_halves(sct_nearest_plan* p, const uint64_t* d_wl, int64_t nw, int G, hipStream_t s) {
  Halves h{};
  h.G = G;
  h.GB = G / 2;
  h.GA = G - h.GB;
  h.nw = nw;
  const int64_t nA = 1LL << (2 * h.GA), nB = 1LL << (2 * h.GB);
  const size_t n = (size_t)std::max<int64_t>(nw, 1);
  int pb = 1;  // bits of a packed whitelist index
  while (pb < 32 && (1LL << pb) < nw) ++pb;
  const int64_t ndw = (2 * (int64_t)n * pb + 31) / 32 + 2;  // + 2: the last 8-byte load's second dword
  // the plan's tables: offA, offB, entA, entB (+16 B: the last chunk's load may run past nw), packed permAB
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t oOffA = 0, oOffB = oOffA + al((nA + 1) * 4), oEntA = oOffB + al((nB + 1) * 4);
  const size_t oEntB = oEntA + al(n * 2 + 16), oPack = oEntB + al(n * 2 + 16), oRank = oPack + al(ndw * 4);
  const size_t total = oRank + al(n);
  SCT_HIP(hipMalloc(&p->hv_mem[0], total));
  char* base = reinterpret_cast<char*>(p->hv_mem[0]);
  h.offA = reinterpret_cast<const uint32_t*>(base + oOffA);
  h.offB = reinterpret_cast<const uint32_t*>(base + oOffB);
  h.entA = reinterpret_cast<const uint16_t*>(base + oEntA);
  h.entB = reinterpret_cast<const uint16_t*>(base + oEntB);
  p->perm_packed = reinterpret_cast<uint32_t*>(base + oPack);
  uint8_t* rankB = reinterpret_cast<uint8_t*>(base + oRank);
  p->pbits = pb;
  // scratch: bucket counts / cursors of both tables, permAB unpacked, the layout flag and the
  // out-of-key-order flag
  const size_t sCnt = 0, sPerm = sCnt + al((nA + nB) * 4), sBad = sPerm + al(2 * n * 4), sTotal = sBad + 256;  // (flags: 1 + kOrders words)
  void* scratch = nullptr;
  SCT_HIP(sct::pool_alloc(&scratch, sTotal, s));
  char* sb = reinterpret_cast<char*>(scratch);
  uint32_t* cntA = reinterpret_cast<uint32_t*>(sb + sCnt);
  uint32_t* cntB = cntA + nA;
  uint32_t* perm = reinterpret_cast<uint32_t*>(sb + sPerm);
  unsigned* bad = reinterpret_cast<unsigned*>(sb + sBad);
  hipError_t e = hipMemsetAsync(sb, 0, sPerm, s);
  if (e == hipSuccess) e = hipMemsetAsync(bad, 0, 4 * (2 + 2 * kOrders), s);
  const unsigned g = grid_for(nw, 4096);
  // the digit order: the first candidate the whitelist is sorted in, chosen on the device (no extra
  // synchronisation; the build's kernels and the host read it from `order`)
  unsigned* order = bad + 1 + kOrders;
  if (e == hipSuccess) {
    if (p->kind == 2)
      hipLaunchKernelGGL(halves_order_kernel<2>, dim3(g), dim3(WG), 0, s, d_wl, nw, h, bad + 1);
    else
      hipLaunchKernelGGL(halves_order_kernel<3>, dim3(g), dim3(WG), 0, s, d_wl, nw, h, bad + 1);
    hipLaunchKernelGGL(halves_pick_order_kernel, dim3(1), dim3(1), 0, s, (const unsigned*)(bad + 1), order);
    e = hipGetLastError();
  }
  if (e == hipSuccess) {
    if (p->kind == 2)
      hipLaunchKernelGGL(halves_count_kernel<2>, dim3(g), dim3(WG), 0, s, d_wl, nw, h, cntA, cntB, bad,
                         (const unsigned*)order);
    else
      hipLaunchKernelGGL(halves_count_kernel<3>, dim3(g), dim3(WG), 0, s, d_wl, nw, h, cntA, cntB, bad,
                         (const unsigned*)order);
    hipLaunchKernelGGL(halves_scan_kernel, dim3(1), dim3(1024), 0, s, cntA, nA, (uint32_t*)h.offA, cntB, nB,
                       (uint32_t*)h.offB);
    if (p->kind == 2)
      hipLaunchKernelGGL(halves_scatter_kernel<2>, dim3(g), dim3(WG), 0, s, d_wl, nw, h, cntA, cntB,
                         (uint16_t*)h.entA, (uint16_t*)h.entB, perm, (const unsigned*)order, rankB,
                         bad + 1 + 2 * kOrders);
    else
      hipLaunchKernelGGL(halves_scatter_kernel<3>, dim3(g), dim3(WG), 0, s, d_wl, nw, h, cntA, cntB,
                         (uint16_t*)h.entA, (uint16_t*)h.entB, perm, (const unsigned*)order, rankB,
                         bad + 1 + 2 * kOrders);
    hipLaunchKernelGGL(pack_perm_kernel, dim3(grid_for(ndw, 4096)), dim3(WG), 0, s, (const uint32_t*)perm,
                       (int64_t)(2 * n), pb, ndw, p->perm_packed);
    e = hipGetLastError();
  }
  // layout not applicable, (unsorted flags), dinv, dalpha, ident_a, an A bucket of > 256 codes
  unsigned hflags[2 + 2 * kOrders] = {1u};
  if (e == hipSuccess) e = hipMemcpyAsync(hflags, bad, sizeof(hflags), hipMemcpyDeviceToHost, s);
  sct::pool_free(scratch, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return sct::fail(SCT_E_HIP, "half-key build: %s", hipGetErrorString(e));
  if (hflags[0]) {  // not applicable: another layout
    (void)hipFree(p->hv_mem[0]);
    p->hv_mem[0] = nullptr;
    p->perm_packed = nullptr;
    return SCT_OK;
  }
  h.dinv = hflags[1 + kOrders];
  h.dalpha = hflags[2 + kOrders];
  h.ident_a = (int)hflags[3 + kOrders];
  h.rankB = h.ident_a && !hflags[1 + 2 * kOrders] ? rankB : nullptr;
  h.perm_packed = p->perm_packed;
  h.pbits = pb;
  p->hv = h;
  p->halves = true;
  return SCT_OK;
}

extern "C" int sct_nearest_plan_create(int kind, const uint64_t* d_whitelist, int64_t nw,
                                       int code_bits, int max_d, void* stream,
                                       sct_nearest_plan** out) {
  SCT_CHECK(out != nullptr, "plan is NULL");
  *out = nullptr;
  SCT_CHECK(kind == 2 || kind == 3, "kind must be 2 or 3");
  SCT_CHECK(nw >= 0 && nw < (1LL << 31), "whitelist size %lld out of range", (long long)nw);
  SCT_CHECK(nw == 0 || d_whitelist != nullptr, "whitelist is NULL");
  SCT_CHECK(code_bits >= 1 && code_bits <= 64, "code_bits %d outside [1, 64]", code_bits);
  const int G = (code_bits + kind - 1) / kind;  // base positions
  SCT_CHECK(max_d >= 0 && max_d + 1 <= MAX_PARTS && max_d < G,
            "max_d %d unsupported (needs max_d+1 <= %d and < %d positions)", max_d, MAX_PARTS, G);
  hipStream_t s = sct::as_stream(stream);
  auto* p = new sct_nearest_plan();
  auto fail_with = [&](int rc) {
    sct_nearest_plan_destroy(p);
    return rc;
  };
  p->kind = kind;
  p->max_d = max_d;
  p->nw = nw;
  p->code_bits = code_bits;
  p->nparts = max_d + 1;
  {
    // half-key tables: max_d <= 1, 2..16 positions, an A/C/G/T whitelist (checked on the device)
    const int64_t forced = sct::tune(SCT_TUNE_NEAREST_SCHEME, 0);
    if ((forced == 0 || forced == SCT_NEAREST_HALVES) && max_d <= 1 && G >= 2 && G <= 16 && nw > 0) {
      if (int rc = build_halves(p, d_whitelist, nw, G, s); rc != SCT_OK) return fail_with(rc);
      if (p->halves) {
        *out = p;
        return SCT_OK;
      }
    }
  }
  sct::DevBuf dup;
  if (dup.alloc((size_t)std::max<int64_t>(nw, 1)) != hipSuccess)
    return fail_with(sct::fail(SCT_E_NOMEM, "dup flags"));
  if (int rc = compute_dups(d_whitelist, nw, (uint8_t*)dup.p, s); rc != SCT_OK) return fail_with(rc);
  // Open addressing when the multi-index keys are nearly unique for random codes: s = 1 block
  // per key for max_d = 0 (the whole code), s = 2 (pairs of P = max_d + 2 blocks) for max_d 1..2,
  // if every key spans enough bases that 4^bases >= nw / 2, i.e. at most ~2 random codes share
  // a key (sct_tune_set(SCT_TUNE_NEAREST_SCHEME, 1 / 2) forces open addressing / CSR).
  {
    const int P = max_d == 0 ? 1 : max_d + 2;
    const int sz = max_d == 0 ? 1 : 2;
    const int nkeys = sz == 1 ? 1 : P * (P - 1) / 2;
    int min_bases = G;  // the smallest key: two smallest blocks of a floor split
    if (sz == 2) min_bases = 2 * (G / P);
    bool oa = P <= G && nkeys <= MAX_KEYS && 2.0 * min_bases >= std::log2(0.5 * std::max<int64_t>(nw, 2));
    const int64_t forced = sct::tune(SCT_TUNE_NEAREST_SCHEME, 0);
    if (forced == SCT_NEAREST_CSR) oa = false;
    if (forced == SCT_NEAREST_OA) oa = P <= G && nkeys <= MAX_KEYS;
    if (oa) {
      uint64_t bmask[MAX_KEYS + 2] = {};
      for (int b = 0; b < P; ++b) {
        const int lo = G * b / P * kind, hi = std::min(64, G * (b + 1) / P * kind);
        bmask[b] = (hi - lo >= 64 ? ~0ull : ((1ull << (hi - lo)) - 1ull)) << lo;
      }
      int64_t nslots = kGroup;
      while (nslots < 2 * nw) nslots *= 2;  // load <= 1/2
      int t = 0;
      for (int a = 0; a < P; ++a)
        for (int b = sz == 1 ? a : a + 1; b < P; ++b) {
          if (sz == 1 && b != a) continue;
          OTable& ot = p->ot.t[t++];
          ot.keymask = bmask[a] | bmask[b];
          ot.gmask = (uint64_t)(nslots / kGroup - 1);
          hipError_t e = hipMalloc(&ot.slots, (size_t)nslots * 16);
          if (e != hipSuccess) return fail_with(sct::fail(SCT_E_NOMEM, "slots: %s", hipGetErrorString(e)));
          hipLaunchKernelGGL(oa_clear_kernel, dim3(grid_for(nslots, 8192)), dim3(WG), 0, s, ot.slots, nslots);
          if (nw)
            hipLaunchKernelGGL(oa_insert_kernel, dim3(grid_for(nw, 4096)), dim3(WG), 0, s, d_whitelist, nw,
                               (const uint8_t*)dup.p, ot);
          SCT_LAUNCH_CHECK();
        }
      p->nkeys = t;
      SCT_HIP(hipStreamSynchronize(s));
      *out = p;
      return SCT_OK;
    }
  }
  // Bucket count per part: a provisional table of ~nw/2 buckets counts the occupied ones
  // (~ the distinct block values: 4^8 = 65,536 for an 8-base ThreeBit block of a 737K
  // whitelist, nw itself for max_d = 0), then the part gets ~SCT_TUNE_NEAREST_LOAD (4) buckets per
  // distinct value, never more than the provisional count: the offset tables stay small
  // enough to live in each XCD's L2 while colliding block values add few extra entries.
  int lg0 = 0;
  while (lg0 < 28 && (1LL << lg0) * 2 < nw) ++lg0;
  const int load = (int)std::max<int64_t>(1, sct::tune(SCT_TUNE_NEAREST_LOAD, 4));
  for (int k = 0; k < p->nparts; ++k) {
    const int pos_lo = G * k / p->nparts, pos_hi = G * (k + 1) / p->nparts;
    Part& pt = p->parts.p[k];
    pt.lo_bit = pos_lo * kind;
    pt.nbits = std::min(64, pos_hi * kind) - pt.lo_bit;
    pt.mask = (pt.nbits >= 64 ? ~0ull : ((1ull << pt.nbits) - 1ull)) << pt.lo_bit;
    pt.mul = lg0 == 0 ? 0ull : 0x9E3779B97F4A7C15ull;
    pt.shift = lg0 == 0 ? 63 : 64 - lg0;
  }
  const int64_t nb0 = 1LL << lg0;
  size_t scan_bytes = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                         (int)(nb0 + 1), s);
  sct::DevBuf scan_tmp, cursor, occ;
  hipError_t e = scan_tmp.alloc(scan_bytes);
  if (e == hipSuccess) e = cursor.alloc((size_t)(nb0 + 1) * 4);
  if (e == hipSuccess) e = occ.alloc(8 * MAX_PARTS);
  if (e != hipSuccess) return fail_with(sct::fail(SCT_E_NOMEM, "scratch: %s", hipGetErrorString(e)));
  uint32_t* counts = (uint32_t*)cursor.p;
  auto* d_occ = (unsigned long long*)occ.p;
  SCT_HIP(hipMemsetAsync(d_occ, 0, 8 * MAX_PARTS, s));
  if (nw && lg0 > 0) {  // occupied provisional buckets per part
    for (int k = 0; k < p->nparts; ++k) {
      SCT_HIP(hipMemsetAsync(counts, 0, (size_t)(nb0 + 1) * 4, s));
      hipLaunchKernelGGL(key_hist_kernel, dim3(grid_for(nw, 4096)), dim3(WG), 0, s, d_whitelist, nw,
                         p->parts.p[k], counts);
      hipLaunchKernelGGL(count_nonzero_kernel, dim3(grid_for(nb0, 1024)), dim3(WG), 0, s, counts, nb0, d_occ + k);
    }
    SCT_LAUNCH_CHECK();
    unsigned long long h_occ[MAX_PARTS] = {};
    SCT_HIP(hipMemcpyAsync(h_occ, d_occ, 8 * MAX_PARTS, hipMemcpyDeviceToHost, s));
    SCT_HIP(hipStreamSynchronize(s));
    for (int k = 0; k < p->nparts; ++k) {
      int lg = 0;
      while (lg < lg0 && (1ULL << lg) < (unsigned long long)load * std::max(1ULL, h_occ[k])) ++lg;
      Part& pt = p->parts.p[k];
      pt.mul = lg == 0 ? 0ull : 0x9E3779B97F4A7C15ull;
      pt.shift = lg == 0 ? 63 : 64 - lg;
      p->nbuckets[k] = 1LL << lg;
    }
  } else {
    for (int k = 0; k < p->nparts; ++k) p->nbuckets[k] = nb0;
  }
  for (int k = 0; k < p->nparts; ++k) {
    const Part pt = p->parts.p[k];
    const int64_t nbuckets = p->nbuckets[k];
    e = hipMalloc(&p->d_off[k], (size_t)(nbuckets + 1) * 4);
    if (e == hipSuccess) e = hipMalloc(&p->d_code[k], (size_t)std::max<int64_t>(nw, 1) * 8);
    if (e == hipSuccess) e = hipMalloc(&p->d_index[k], (size_t)std::max<int64_t>(nw, 1) * 4);
    if (e != hipSuccess) return fail_with(sct::fail(SCT_E_NOMEM, "bucket arrays: %s", hipGetErrorString(e)));
    SCT_HIP(hipMemsetAsync(counts, 0, (size_t)(nbuckets + 1) * 4, s));
    if (nw)
      hipLaunchKernelGGL(key_hist_kernel, dim3(grid_for(nw, 4096)), dim3(WG), 0, s, d_whitelist, nw,
                         pt, counts);
    size_t b = scan_bytes;
    e = hipcub::DeviceScan::ExclusiveSum(scan_tmp.p, b, counts, p->d_off[k], (int)(nbuckets + 1), s);
    if (e != hipSuccess) return fail_with(sct::fail(SCT_E_HIP, "scan: %s", hipGetErrorString(e)));
    SCT_HIP(hipMemcpyAsync(counts, p->d_off[k], (size_t)nbuckets * 4, hipMemcpyDeviceToDevice, s));
    if (nw)
      hipLaunchKernelGGL(key_scatter_kernel, dim3(grid_for(nw, 4096)), dim3(WG), 0, s, d_whitelist,
                         nw, pt, counts, (const uint8_t*)dup.p, p->d_code[k], p->d_index[k]);
    SCT_LAUNCH_CHECK();
  }
  SCT_HIP(hipStreamSynchronize(s));  // the scratch buffers die with this call
  *out = p;
  return SCT_OK;
}

extern "C" int sct_nearest_plan_info(const sct_nearest_plan* p, int* scheme, int64_t* index_bytes) {
  SCT_CHECK(p != nullptr, "plan is NULL");
  int64_t bytes = 0;
  if (p->halves) {
    bytes = ((1LL << (2 * p->hv.GA)) + (1LL << (2 * p->hv.GB)) + 2) * 4 + p->nw * 4 + (2 * p->nw * p->pbits + 31) / 32 * 4;
    if (scheme) *scheme = SCT_NEAREST_HALVES;
    if (index_bytes) *index_bytes = bytes;
    return SCT_OK;
  }
  if (p->nkeys > 0) {
    for (int k = 0; k < p->nkeys; ++k) bytes += (int64_t)(p->ot.t[k].gmask + 1) * kGroup * 16;
  } else {
    for (int k = 0; k < p->nparts; ++k) bytes += (p->nbuckets[k] + 1) * 4 + p->nw * 12;
  }
  if (scheme) *scheme = p->nkeys > 0 ? SCT_NEAREST_OA : SCT_NEAREST_CSR;
  if (index_bytes) *index_bytes = bytes;
  return SCT_OK;
}

static int nearest_query_launch(sct_nearest_plan* p, const uint64_t* d_queries, int64_t nq, int32_t* d_index,
                                uint8_t* d_dist, void* stream);

extern "C" int sct_nearest_query(sct_nearest_plan* p, const uint64_t* d_queries, int64_t nq,
                                 int32_t* d_index, uint8_t* d_dist, void* stream) {
  const int rc = nearest_query_launch(p, d_queries, nq, d_index, d_dist, stream);
  if (rc == SCT_OK && p && nq > 0) {
    if (!p->last_query) SCT_HIP(hipEventCreateWithFlags(&p->last_query, hipEventDisableTiming));
    SCT_HIP(hipEventRecord(p->last_query, sct::as_stream(stream)));
  }
  return rc;
}

static int nearest_query_launch(sct_nearest_plan* p, const uint64_t* d_queries, int64_t nq, int32_t* d_index,
                                uint8_t* d_dist, void* stream) {
  SCT_CHECK(p != nullptr, "plan is NULL");
  SCT_CHECK(nq >= 0, "nq must be >= 0");
  if (nq == 0) return SCT_OK;
  SCT_CHECK(d_queries && d_index && d_dist, "NULL pointer");
  hipStream_t s = sct::as_stream(stream);
  const unsigned blocks = (unsigned)sct::ceil_div(nq, WG);  // one query per thread
  SCT_CHECK(sct::ceil_div(nq, WG) < (1LL << 31), "too many queries for one launch");
  if (p->halves) {
    if (p->hv.ident_a) {  // whitelist indices straight from the query kernel
      auto kern = p->kind == 2 ? halves_query_kernel<2, true> : halves_query_kernel<3, true>;
      hipLaunchKernelGGL(kern, dim3(blocks), dim3(WG), 0, s, d_queries, nq, p->hv, p->max_d, d_index, d_dist);
      SCT_LAUNCH_CHECK();
      return SCT_OK;
    }
    auto kern = p->kind == 2 ? halves_query_kernel<2, false> : halves_query_kernel<3, false>;
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(WG), 0, s, d_queries, nq, p->hv, p->max_d, d_index, d_dist);
    SCT_LAUNCH_CHECK();
    hipLaunchKernelGGL(halves_index_kernel, dim3(grid_for(sct::ceil_div(nq, 4), 8192)), dim3(WG), 0, s, d_index, nq,
                       (const uint32_t*)p->perm_packed, p->pbits, ((uintptr_t)d_index & 15) == 0);
    SCT_LAUNCH_CHECK();
    return SCT_OK;
  }
  if (p->nkeys > 0) {
    if (p->kind == 2)
      launch_oa_query<2>(p->nkeys, blocks, s, d_queries, nq, p->ot, p->max_d, d_index, d_dist);
    else
      launch_oa_query<3>(p->nkeys, blocks, s, d_queries, nq, p->ot, p->max_d, d_index, d_dist);
    SCT_LAUNCH_CHECK();
    return SCT_OK;
  }
  Tables tb{};
  for (int k = 0; k < p->nparts; ++k) {
    tb.part[k] = p->parts.p[k];
    tb.off[k] = p->d_off[k];
    tb.code[k] = p->d_code[k];
    tb.index[k] = p->d_index[k];
  }
  if (p->kind == 2)
    launch_query<2>(p->nparts, blocks, s, d_queries, nq, tb, p->max_d, d_index, d_dist);
  else
    launch_query<3>(p->nparts, blocks, s, d_queries, nq, tb, p->max_d, d_index, d_dist);
  SCT_LAUNCH_CHECK();
  return SCT_OK;
}

extern "C" int sct_nearest_host(int kind, const uint64_t* whitelist, int64_t nw, const uint64_t* queries,
                                int64_t nq, int code_bits, int max_d, int32_t* index, uint8_t* dist) {
  SCT_CHECK(nw >= 0 && nq >= 0, "bad sizes");
  // a host-whitelist plan and one host query pass (both through the library's stream-ordered
  // pool on the thread's stream: no per-call hipMalloc / hipFree); the results are read back
  // before the plan goes
  sct_nearest_plan* plan = nullptr;
  int rc = sct_nearest_plan_create_host(kind, whitelist, nw, code_bits, max_d, &plan);
  if (rc != SCT_OK) return rc;
  rc = sct_nearest_query_host(plan, queries, nq, index, dist);
  sct_nearest_plan_destroy(plan);
  return rc;
}

extern "C" int sct_nearest_plan_create_host(int kind, const uint64_t* whitelist, int64_t nw, int code_bits, int max_d,
                                            sct_nearest_plan** out) {
  SCT_CHECK(out != nullptr, "plan is NULL");
  SCT_CHECK(nw >= 0 && (nw == 0 || whitelist), "bad whitelist");
  // the whitelist through the library's stream-ordered pool on the thread's stream (no per-call
  // hipMalloc / hipFree: a stream of batches builds its index once, but the flows that build
  // one per file set pay it each time)
  sct::HostStage* hs = sct::host_stage();
  if (!hs) return SCT_E_HIP;
  hipStream_t s = hs->stream;
  void* dw = nullptr;
  SCT_HIP(sct::pool_alloc(&dw, std::max<size_t>((size_t)nw * 8, 8), s));
  hipError_t e = nw ? hipMemcpyAsync(dw, whitelist, (size_t)nw * 8, hipMemcpyHostToDevice, s) : hipSuccess;
  int rc = e == hipSuccess ? sct_nearest_plan_create(kind, (const uint64_t*)dw, nw, code_bits, max_d, s, out)
                           : sct::fail(SCT_E_HIP, "whitelist copy: %s", hipGetErrorString(e));
  sct::pool_free(dw, s);  // (ordered after the build's reads of it)
  e = hipStreamSynchronize(s);
  if (rc == SCT_OK && e != hipSuccess) rc = sct::fail(SCT_E_HIP, "nearest plan: %s", hipGetErrorString(e));
  return rc;
}

extern "C" int sct_nearest_query_host(sct_nearest_plan* p, const uint64_t* queries, int64_t nq, int32_t* index,
                                      uint8_t* dist) {
  SCT_CHECK(p != nullptr, "plan is NULL");
  SCT_CHECK(nq >= 0 && (nq == 0 || (queries && index && dist)), "bad arguments");
  if (nq == 0) return SCT_OK;
  sct::HostStage* hs = sct::host_stage();
  if (!hs) return SCT_E_HIP;
  hipStream_t s = hs->stream;
  const size_t qb = ((size_t)nq * 8 + 255) & ~(size_t)255, ib = ((size_t)nq * 4 + 255) & ~(size_t)255;
  void* blk = nullptr;
  SCT_HIP(sct::pool_alloc(&blk, qb + ib + (size_t)nq, s));
  uint8_t* b = static_cast<uint8_t*>(blk);
  int rc = SCT_OK;
  hipError_t e = hipMemcpyAsync(b, queries, (size_t)nq * 8, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) {
    rc = sct_nearest_query(p, (const uint64_t*)b, nq, (int32_t*)(b + qb), b + qb + ib, s);
    if (rc == SCT_OK) {
      e = hipMemcpyAsync(index, b + qb, (size_t)nq * 4, hipMemcpyDeviceToHost, s);
      if (e == hipSuccess) e = hipMemcpyAsync(dist, b + qb + ib, (size_t)nq, hipMemcpyDeviceToHost, s);
    }
  }
  sct::pool_free(blk, s);
  const hipError_t se = hipStreamSynchronize(s);
  if (e == hipSuccess) e = se;
  if (rc == SCT_OK && e != hipSuccess) rc = sct::fail(SCT_E_HIP, "nearest query: %s", hipGetErrorString(e));
  return rc;
}
