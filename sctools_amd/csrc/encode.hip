// Element-wise encoding kernels for gfx950: encode (TwoBit/ThreeBit + GC + flags),
// decode, gc_content and pairwise Hamming distance.  All are one-record-per-lane,
// HBM-bound streaming kernels; the byte->code map is a 256-entry LDS table.
//
// Reference semantics (src/sctools/encodings.py):
//   TwoBit map      :53-69   A/a 0, C/c 1, T/t 2, G/g 3; IUPAC ambiguity -> random
//                            (flagged here, drawn by the Python caller in order);
//                            anything else -> KeyError (flagged here)
//   TwoBit.encode   :75-88   MSB-first, 2 bits per byte
//   TwoBit.decode   :90-100  exactly L bases from the LSB upward
//   TwoBit.gc       :102-111 low bit of each of the L groups
//   TwoBit.hamming  :113-121 non-zero 2-bit groups of a^b
//   ThreeBit map    :139-149 C 1, A 2, G 3, T 4, N 6, any other byte -> 6
//   ThreeBit.encode :155-167 MSB-first, 3 bits per byte
//   ThreeBit.decode :169-180 triplets up to the top non-zero one; 0/5/7 -> KeyError
//   ThreeBit.gc     :182-192 bit 0 of every triplet
//   ThreeBit.hamming:194-202 non-zero 3-bit groups of a^b
#include <stddef.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>
#include <vector>

#include "sct_common.h"
#include "encode_common.h"

namespace {

constexpr int WG = 256;
__device__ __forceinline__ void fill_lut(uint8_t* lut, int kind) {
  for (int c = threadIdx.x; c < 256; c += blockDim.x) lut[c] = lut_entry(kind, c);
  __syncthreads();
}

// Records at seqs + r * stride of L bytes, or (starts != nullptr) at seqs + starts[r] of
// lens[r] bytes each (variable-length lines: the whitelist ingest, sctools_amd/csrc/lines.hip).
__global__ __launch_bounds__(WG) void encode_kernel(int kind, const uint8_t* __restrict__ seqs,
                                                    int64_t n, int64_t stride, int L_all, int words,
                                                    bool dword_path, uint64_t* __restrict__ codes,
                                                    uint8_t* __restrict__ gc,
                                                    uint8_t* __restrict__ flags,
                                                    const int64_t* __restrict__ starts = nullptr,
                                                    const int32_t* __restrict__ lens = nullptr) {
  __shared__ uint8_t lut[256];
  fill_lut(lut, kind);
  for (int64_t r = (int64_t)blockIdx.x * WG + threadIdx.x; r < n; r += (int64_t)gridDim.x * WG) {
    const int L = starts ? lens[r] : L_all;
    RecordReader rd{seqs + (starts ? starts[r] : r * stride), dword_path, 0u, -1};
    uint32_t g, fl;
    encode_record(lut, kind, rd, L, words, codes + r * words, g, fl);
    if (gc) gc[r] = (uint8_t)(g > 255 ? 255 : g);
    if (flags) flags[r] = (uint8_t)fl;
  }
}

// Variable-length records of one limb (the whitelist's lines): each lane loads the aligned
// dwords that hold its record (at most 9 for 32 bases: every load independent, and a wave's
// loads of consecutive lines cover consecutive lines of memory), realigns them by the start's
// byte offset and reads every position's LUT entry independently.  Only dwords holding a byte
// of the record are loaded, so no load leaves the pages the record lies in.  Records longer
// than 32 bytes take the byte loop.
__global__ __launch_bounds__(WG) void encode_var_kernel(int kind, const uint8_t* __restrict__ buf, int64_t n,
                                                        const int64_t* __restrict__ starts,
                                                        const int32_t* __restrict__ lens,
                                                        uint64_t* __restrict__ codes, uint8_t* __restrict__ gc,
                                                        uint8_t* __restrict__ flags) {
  __shared__ uint8_t lut[256];
  fill_lut(lut, kind);
  const uint64_t gcm = kind == 2 ? 0x5555555555555555ull : 0x9249249249249249ull;
  for (int64_t r = (int64_t)blockIdx.x * WG + threadIdx.x; r < n; r += (int64_t)gridDim.x * WG) {
    const uint8_t* rec = buf + starts[r];
    const int L = lens[r];
    uint64_t code = 0;
    uint32_t fl = 0;
    if (L == 0) {
    } else if (L <= 32) {
      const int o = (int)((uintptr_t)rec & 3), o8 = 8 * o;
      const uint32_t* dw = reinterpret_cast<const uint32_t*>(rec - o);
      uint32_t d[9], w[8];
#pragma unroll
      for (int k = 0; k < 9; ++k) {  // dword k of the record, clamped to its last one (no branch)
        const int kk = 4 * k < o + L ? k : (o + L - 1) >> 2;
        d[k] = __builtin_nontemporal_load(dw + kk);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) w[k] = (uint32_t)((((uint64_t)d[k + 1] << 32) | d[k]) >> o8);
#pragma unroll
      for (int p = 0; p < 32; ++p)
        if (p < L) {
          const uint32_t e = lut[(w[p >> 2] >> (8 * (p & 3))) & 0xFFu];
          code = (code << kind) | (e & 7u);
          fl |= e;
        }
    } else {
      for (int p = 0; p < L; ++p) {
        const uint32_t e = lut[rec[p]];
        code = (code << kind) | (e & 7u);
        fl |= e;
      }
    }
    codes[r] = code;
    if (gc) {
      const uint32_t g = (uint32_t)__popcll(code & gcm);
      gc[r] = (uint8_t)(g > 255 ? 255 : g);
    }
    if (flags) flags[r] = (uint8_t)(((fl & F_AMBIG) ? 1u : 0u) | ((fl & F_INVALID) ? 2u : 0u));
  }
}

// Contiguous records (stride == L, one limb): a workgroup stages 256 records with
// coalesced 16-byte loads into LDS, then each lane packs its record from LDS (dword reads
// when L % 4 == 0, conflict-free for odd L/4) through the LDS byte LUT.  The staging
// turns the per-lane, L-byte-strided global loads of encode_kernel into full-line reads.
template <int BITS, int R>
__global__ __launch_bounds__(WG) void encode_tiled_kernel(const uint8_t* __restrict__ seqs,
                                                          int64_t n, int L,
                                                          uint64_t* __restrict__ codes,
                                                          uint8_t* __restrict__ gc,
                                                          uint8_t* __restrict__ flags) {
  __shared__ uint8_t lut[256];
  extern __shared__ __attribute__((aligned(16))) uint4 stage4[];  // R * WG * L bytes
  fill_lut(lut, BITS);
  const uint8_t* stage = reinterpret_cast<const uint8_t*>(stage4);
  const int tid = threadIdx.x;
  constexpr int TILE = R * WG;  // records per workgroup iteration: R in flight per lane
  const int64_t ntiles = (n + TILE - 1) / TILE;
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
  // a thread's 16-B loads of a tile are all issued before any of them is stored to LDS (8
  // per batch: 7 at L = 28).  When one batch holds a whole tile (L * R <= 128) the next
  // tile's loads are issued right after this tile's LDS stores, so they fly while this
  // tile is packed.
  const bool pipe = L * R <= 128;
  v4u t[8];
  auto fetch = [&](int64_t tl, int64_t k0) {
    const int64_t rb = tl * TILE, nr = n - rb < TILE ? n - rb : TILE;
    const int64_t m16 = (nr * L) >> 4;
    const v4u* s4 = reinterpret_cast<const v4u*>(seqs + rb * L);  // 16-B aligned: TILE * L % 16 == 0
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t k = k0 + u * WG + tid;
      if (k < m16) t[u] = __builtin_nontemporal_load(s4 + k);
    }
  };
  if (pipe && (int64_t)blockIdx.x < ntiles) fetch(blockIdx.x, 0);
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t r0 = tile * TILE;
    const int64_t nrec = n - r0 < TILE ? n - r0 : TILE;
    const int64_t nbytes = nrec * L;
    const uint8_t* src = seqs + r0 * L;
    const int64_t n16 = nbytes >> 4;
    for (int64_t k0 = 0; k0 < n16; k0 += 8 * WG) {
      if (!pipe) fetch(tile, k0);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int64_t k = k0 + u * WG + tid;
        if (k < n16) stage4[k] = make_uint4(t[u].x, t[u].y, t[u].z, t[u].w);
      }
    }
    if (pipe && tile + gridDim.x < ntiles) fetch(tile + gridDim.x, 0);
    for (int64_t k = (n16 << 4) + tid; k < nbytes; k += WG)
      reinterpret_cast<uint8_t*>(stage4)[k] = src[k];
    __syncthreads();
#pragma unroll
    for (int rr = 0; rr < R; ++rr) {
      const int lr = rr * WG + tid;  // consecutive lanes -> consecutive records (coalesced stores)
      if (lr < nrec) {
        const uint8_t* rec = stage + (int64_t)lr * L;
        uint64_t code = 0;
        uint32_t fl = 0;
        bool done = false;
        if (BITS == 2 && (L & 3) == 0) {
          // TwoBit, 4 bases per dword without the LUT: u = the bytes upper-cased; their low 3
          // bits (A 1, C 3, T 4, G 7) index a v_perm byte table of the expected letters, so
          // u == table[u & 7] in every byte iff all four are ACGTacgt.  The values are
          // (u >> 1) & 3 per byte (A 0, C 1, T 2, G 3), gathered MSB-first into one byte by
          // one multiply: v * (1 + 2^10 + 2^20 + 2^30) puts byte j's value at bits 30 - 2j,
          // every other partial product in a disjoint 2-bit slot below 24 (no carries).
          // A byte that is not a base (N, IUPAC, invalid: 1 % of config 5's reads) has code bits
          // 0 (lut & 7 for every such byte), so it is cleared through the byte mask of the
          // mismatch and only its flag is read from the LUT -- every lane runs the same steps
          // (the divergent 28-step LUT loop this replaces cost 1.2 ms of 7.8 on config 5's 1e9
          // reads: half the waves carried a read with an N).  One limb: L <= 32, <= 8 dwords.
          const uint32_t* rw = reinterpret_cast<const uint32_t*>(rec);
          uint32_t nzs[8], anyb = 0;
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            nzs[k] = 0;
            if (k < (L >> 2)) {
              const uint32_t u = rw[k] & 0xDFDFDFDFu;
              const uint32_t d = u ^ __builtin_amdgcn_perm(0x47010154u, 0x43014101u, u & 0x07070707u);
              const uint32_t nz = (((d & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | d) & 0x80808080u;  // bit 7: differs
              const uint32_t v = ((u >> 1) & 0x03030303u) & ~((nz - (nz >> 7)) | nz);
              code = (code << 8) | ((v * 0x40100401u) >> 24);
              nzs[k] = nz;
              anyb |= nz;
            }
          }
          if (anyb) {
#pragma unroll
            for (int k = 0; k < 8; ++k)
              for (uint32_t b = nzs[k]; b; b &= b - 1) fl |= lut[(rw[k] >> (__builtin_ctz(b) - 7)) & 0xFFu];
          }
          done = true;
        }
        if (done) {
        } else if ((L & 3) == 0) {
          const uint32_t* rw = reinterpret_cast<const uint32_t*>(rec);
          for (int k = 0; k < (L >> 2); ++k) {
            const uint32_t w = rw[k];
#pragma unroll
            for (int b = 0; b < 4; ++b) {
              const uint32_t e = lut[(w >> (8 * b)) & 0xFFu];
              code = (code << BITS) | (e & 7u);
              fl |= e;
            }
          }
        } else {
          for (int p = 0; p < L; ++p) {
            const uint32_t e = lut[rec[p]];
            code = (code << BITS) | (e & 7u);
            fl |= e;
          }
        }
        const int64_t r = r0 + lr;
        codes[r] = code;
        if (gc)
          gc[r] = (uint8_t)__popcll(code & (BITS == 2 ? 0x5555555555555555ull : 0x9249249249249249ull));
        if (flags) flags[r] = (uint8_t)(((fl & F_AMBIG) ? 1u : 0u) | ((fl & F_INVALID) ? 2u : 0u));
      }
    }
    __syncthreads();
  }
}

__device__ __forceinline__ uint64_t limb(const uint64_t* w, int words, int i) {
  return i < words ? w[i] : 0ull;
}

// value of the `width`-bit group starting at bit `pos` of a multi-limb integer
__device__ __forceinline__ uint32_t group_at(const uint64_t* w, int words, int64_t pos, int width) {
  const int i = (int)(pos >> 6), off = (int)(pos & 63);
  uint64_t v = limb(w, words, i) >> off;
  if (off + width > 64) v |= limb(w, words, i + 1) << (64 - off);
  return (uint32_t)(v & ((1u << width) - 1u));
}

__device__ __forceinline__ void decode2_limbs(const uint64_t* w, int words, int L, uint8_t* o) {
  for (int p = 0; p < L; ++p) {
    const int64_t pos = 2LL * (L - 1 - p);
    const uint32_t v = pos < 64LL * words ? group_at(w, words, pos, 2) : 0u;
    // "ACTG"[v] from a register (the string literal was a global load per base: ~2 us of a
    // 16-base scalar decode)
    o[p] = (uint8_t)(0x47544341u >> (8 * v));
  }
}

// A one-limb code is read once into a register and its bases leave four to a store: through the
// generic path the byte stores to o (which may alias w) made the compiler reload the code for
// every base, one dependent LDS read each in the scalar server (85 ns per base per call)
__device__ __forceinline__ void decode2_record(const uint64_t* w, int words, int L, uint8_t* o) {
  if (words != 1) {
    decode2_limbs(w, words, L, o);
    return;
  }
  const uint64_t c = w[0];
  auto base = [&](int p) {  // "ACTG"[group L-1-p], 'A' above the limb
    const int pos = 2 * (L - 1 - p);
    const uint32_t v = pos < 64 ? (uint32_t)(c >> pos) & 3u : 0u;
    return (0x47544341u >> (8 * v)) & 0xFFu;
  };
  int p = 0;
  if (((uintptr_t)o & 3u) == 0u)
    for (; p + 4 <= L; p += 4)
      *reinterpret_cast<uint32_t*>(o + p) = base(p) | base(p + 1) << 8 | base(p + 2) << 16 | base(p + 3) << 24;
  for (; p < L; ++p) o[p] = (uint8_t)base(p);
}

__global__ __launch_bounds__(WG) void decode2_kernel(const uint64_t* __restrict__ codes, int64_t n,
                                                     int words, int L, uint8_t* __restrict__ out) {
  for (int64_t r = (int64_t)blockIdx.x * WG + threadIdx.x; r < n; r += (int64_t)gridDim.x * WG)
    decode2_record(codes + r * words, words, L, out + r * L);
}

// o[maxlen - 1 - t] = base of triplet t for t <= the top non-zero triplet; returns that
// count, and in err the first invalid triplet value (0 / 5 / 7) or -1
__device__ __forceinline__ int32_t decode3_limbs(const uint64_t* w, int words, int maxlen, uint8_t* o,
                                                 int32_t& err) {
  const int ntrip = (64 * words + 2) / 3;
  int top = -1;
  for (int t = ntrip - 1; t >= 0; --t)
    if (group_at(w, words, 3LL * t, 3) != 0u) {
      top = t;
      break;
    }
  err = -1;
  for (int t = 0; t <= top; ++t) {
    const uint32_t v = group_at(w, words, 3LL * t, 3);
    uint8_t ch = 0;
    switch (v) {
      case 1: ch = 'C'; break;
      case 2: ch = 'A'; break;
      case 3: ch = 'G'; break;
      case 4: ch = 'T'; break;
      case 6: ch = 'N'; break;
      default:
        if (err < 0) err = (int32_t)v;
        break;
    }
    o[maxlen - 1 - t] = ch;
  }
  return top + 1;
}

// (a one-limb code in a register, as decode2_record)
__device__ __forceinline__ int32_t decode3_record(const uint64_t* w, int words, int maxlen, uint8_t* o,
                                                  int32_t& err) {
  if (words != 1) return decode3_limbs(w, words, maxlen, o, err);
  const uint64_t c = w[0];
  const int top = c ? (63 - __clzll((long long)c)) / 3 : -1;  // the top non-zero triplet
  err = -1;
  for (int t = 0; t <= top; ++t) {
    const uint32_t v = (uint32_t)(c >> (3 * t)) & 7u;
    // C A G T at 1..4, N at 6 (bytes of 0x544741434E: v = 1..4 -> byte v - 1, 6 -> byte 4)
    const bool ok = (v >= 1u && v <= 4u) || v == 6u;
    if (!ok && err < 0) err = (int32_t)v;
    o[maxlen - 1 - t] = ok ? (uint8_t)(0x4E54474143ull >> (8 * (v == 6u ? 4u : v - 1u))) : (uint8_t)0;
  }
  return top + 1;
}

__global__ __launch_bounds__(WG) void decode3_kernel(const uint64_t* __restrict__ codes, int64_t n,
                                                     int words, int maxlen, uint8_t* __restrict__ out,
                                                     int32_t* __restrict__ lengths,
                                                     int32_t* __restrict__ bad) {
  for (int64_t r = (int64_t)blockIdx.x * WG + threadIdx.x; r < n; r += (int64_t)gridDim.x * WG) {
    int32_t err;
    lengths[r] = decode3_record(codes + r * words, words, maxlen, out + r * maxlen, err);
    bad[r] = err;
  }
}

// bit-0-of-each-triplet mask for limb i (64*i mod 3 shifts the pattern)
__device__ __forceinline__ uint64_t m3(int i) {
  switch (i % 3) {
    case 0: return 0x9249249249249249ull;
    case 1: return 0x4924924924924924ull;
    default: return 0x2492492492492492ull;
  }
}

__device__ __forceinline__ int32_t gc_record(int kind, const uint64_t* w, int words, int L) {
  int32_t g = 0;
  for (int i = 0; i < words; ++i) {
    uint64_t m;
    if (kind == 2) {
      const int64_t lo = 64LL * i, rem = 2LL * L - lo;  // bits of the L groups inside this limb
      if (rem <= 0) break;
      m = 0x5555555555555555ull;
      if (rem < 64) m &= (1ull << rem) - 1ull;
    } else {
      m = m3(i);
    }
    g += __popcll(w[i] & m);
  }
  return g;
}

__global__ __launch_bounds__(WG) void gc_kernel(int kind, const uint64_t* __restrict__ codes,
                                                int64_t n, int words, int L,
                                                int32_t* __restrict__ out) {
  for (int64_t r = (int64_t)blockIdx.x * WG + threadIdx.x; r < n; r += (int64_t)gridDim.x * WG)
    out[r] = gc_record(kind, codes + r * words, words, L);
}

__device__ __forceinline__ int32_t hamming_record(int kind, const uint64_t* x, const uint64_t* y, int words) {
  int32_t d = 0;
  if (kind == 2) {
    for (int i = 0; i < words; ++i) {
      const uint64_t v = x[i] ^ y[i];
      d += __popcll((v | (v >> 1)) & 0x5555555555555555ull);
    }
  } else {
    uint64_t v = x[0] ^ y[0];
    for (int i = 0; i < words; ++i) {
      const uint64_t nx = i + 1 < words ? (x[i + 1] ^ y[i + 1]) : 0ull;
      const uint64_t s = v | ((v >> 1) | (nx << 63)) | ((v >> 2) | (nx << 62));
      d += __popcll(s & m3(i));
      v = nx;
    }
  }
  return d;
}

__global__ __launch_bounds__(WG) void hamming_kernel(int kind, const uint64_t* __restrict__ a,
                                                     const uint64_t* __restrict__ b, int64_t n,
                                                     int words, int32_t* __restrict__ out) {
  for (int64_t r = (int64_t)blockIdx.x * WG + threadIdx.x; r < n; r += (int64_t)gridDim.x * WG)
    out[r] = hamming_record(kind, a + r * words, b + r * words, words);
}

// Per-position base counts.  Base p of a code is bits 2j, 2j + 1 with j = L - 1 - p, and only
// j < 32 can be non-zero, so the work is the 32 2-bit fields j of the codes, counted in
// registers with SWAR counters (no per-code atomics, no per-field loop): per code the
// indicator masks of values 1, 2, 3 (bit 2j set when field j holds that value) are added into
// nibble counters (fields 2i / 2i + 1 in nibble i of two words), folded every 15 codes into
// byte counters (field 4k + q in byte k of word q), and those, every 255 codes or at the end,
// are widened to 16-bit lanes, summed over the wave by shuffles and added to the workgroup's
// LDS tally.  Each workgroup writes its 128 partials (bin-major), which
// base_frequency_reduce_kernel sums: no same-address global atomics.  A lane's codes are
// gridDim * 256 apart, so a wave's loads stay coalesced.
__global__ __launch_bounds__(WG) void base_frequency_kernel(const uint64_t* __restrict__ codes,
                                                            int64_t n, unsigned long long* __restrict__ part) {
  constexpr uint64_t K5 = 0x5555555555555555ull, K1 = 0x1111111111111111ull, KF = 0x0F0F0F0F0F0F0F0Full;
  __shared__ unsigned long long tally[32][4];
  const int tid = threadIdx.x, lane = tid & 63;
  if (tid < 128) tally[tid >> 2][tid & 3] = 0;
  __syncthreads();
  const int64_t G = (int64_t)gridDim.x * WG;
  unsigned long long seen = 0;
  for (int64_t e0 = (int64_t)blockIdx.x * WG + tid; e0 - tid < n; e0 += 255 * G) {  // epochs of <= 255 codes per lane
    uint64_t Q[3][4] = {};  // [value - 1][q]: byte k counts field 4k + q
    for (int c = 0; c < 17; ++c) {
      const int64_t c0 = e0 + (int64_t)c * 15 * G;
      if (c0 - tid >= n) break;  // workgroup-uniform
      uint64_t N[3][2] = {};  // [value - 1][field parity]: nibble i counts field 2i + parity
      uint64_t xs[15];
#pragma unroll
      for (int u = 0; u < 15; ++u) {  // all 15 loads issued first (clamped, not branched around)
        const int64_t r = c0 + u * G;
        xs[u] = codes[r < n ? r : n - 1];
      }
#pragma unroll
      for (int u = 0; u < 15; ++u) {
        const int64_t r = c0 + u * G;
        if (r < n) {
          const uint64_t x = xs[u];
          const uint64_t lo = x & K5, hi = (x >> 1) & K5, m3 = lo & hi, m[3] = {lo ^ m3, hi ^ m3, m3};
#pragma unroll
          for (int v = 0; v < 3; ++v) {
            N[v][0] += m[v] & K1;
            N[v][1] += (m[v] >> 2) & K1;
          }
          ++seen;
        }
      }
#pragma unroll
      for (int v = 0; v < 3; ++v) {
        Q[v][0] += N[v][0] & KF;         // fields 4k
        Q[v][2] += (N[v][0] >> 4) & KF;  // fields 4k + 2
        Q[v][1] += N[v][1] & KF;         // fields 4k + 1
        Q[v][3] += (N[v][1] >> 4) & KF;  // fields 4k + 3
      }
    }
    // bytes -> 16-bit lanes (even / odd bytes), summed over the wave (<= 64 * 255 per lane)
#pragma unroll
    for (int v = 0; v < 3; ++v)
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          uint64_t w = (Q[v][q] >> (8 * h)) & 0x00FF00FF00FF00FFull;  // u16 lane i = byte 2i + h
#pragma unroll
          for (int o = 32; o; o >>= 1) w += __shfl_xor(w, o);
          if (lane < 4) {  // lane i takes u16 lane i: byte k = 2i + h, field 4k + q
            const int k = 2 * lane + h;
            atomicAdd(&tally[4 * k + q][v + 1], (unsigned long long)((w >> (16 * lane)) & 0xFFFFu));
          }
        }
  }
  for (int o = 32; o; o >>= 1) seen += __shfl_xor(seen, o);
  if (lane == 0) atomicAdd(&tally[0][0], seen);  // codes seen; value 0 = seen - the rest
  __syncthreads();
  if (tid < 128) {
    const int j = tid >> 2, v = tid & 3;
    unsigned long long t = tally[j][v];
    if (v == 0) t = tally[0][0] - tally[j][1] - tally[j][2] - tally[j][3];
    part[(size_t)tid * gridDim.x + blockIdx.x] = t;
  }
}

// L <= 16 (every output field j < 16 lies in a code's low 32 bits; the bits above are never
// read): the same partials from 32-bit words at a third of the instructions.  Per code the
// indicator masks m_v (bit 2j set when field j holds v = 1..3) come from x and x >> 1 by one
// bitop3 each; three codes' masks add in one v_add3_u32 (2-bit fields, <= 3), five such sums
// into nibble counters (fields 2i / 2i + 1 in nibble i of two words, <= 15), then into byte
// counters (field 4k + {0, 2, 1, 3}[w] in byte k of word w).  The host sizes the grid so no
// lane sees more than 255 codes.  The workgroup's 12 x 256 byte-counter words meet in LDS and
// 192 threads sum them (byte pairs widened to 16-bit lanes, <= 256 * 255), so the epilogue is
// 16 LDS reads and 8 shuffles per thread instead of 24 64-bit wave reductions per wave.
__global__ __launch_bounds__(WG) void base_frequency16_kernel(const uint64_t* __restrict__ codes, int64_t n,
                                                              unsigned long long* __restrict__ part) {
  constexpr uint32_t K5 = 0x55555555u, K3 = 0x33333333u, KF = 0x0F0F0F0Fu;
  __shared__ uint32_t xch[WG / 64][12][64];
  __shared__ uint32_t cnt[16][4];  // [field j][value v]
  __shared__ uint32_t seen_w[WG / 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t G = (int64_t)gridDim.x * WG;
  const uint32_t* lo32 = reinterpret_cast<const uint32_t*>(codes);  // (little endian: word 2r = low half)
  uint32_t B[3][4] = {};
  uint32_t seen = 0;
  for (int64_t c0 = (int64_t)blockIdx.x * WG + tid; c0 - tid < n; c0 += 15 * G) {  // rounds of 15 codes
    uint32_t xs[15];
#pragma unroll
    for (int u = 0; u < 15; ++u) {  // all 15 loads issued first (clamped, then zeroed: a zero adds no mask)
      const int64_t r = c0 + u * G;
      xs[u] = lo32[2 * (r < n ? r : n - 1)];
    }
#pragma unroll
    for (int u = 0; u < 15; ++u) {
      const bool in = c0 + u * G < n;
      xs[u] = in ? xs[u] : 0u;
      seen += in ? 1u : 0u;
    }
    uint32_t Ne[3] = {0, 0, 0}, No[3] = {0, 0, 0};
#pragma unroll
    for (int g = 0; g < 5; ++g) {
      uint32_t m[3][3];
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const uint32_t x = xs[3 * g + t], y = x >> 1;
        m[0][t] = x & ~y & K5;  // 01: value 1
        m[1][t] = ~x & y & K5;  // 10: value 2
        m[2][t] = x & y & K5;   // 11: value 3
      }
#pragma unroll
      for (int v = 0; v < 3; ++v) {
        const uint32_t S = m[v][0] + m[v][1] + m[v][2];
        Ne[v] += S & K3;
        No[v] += (S >> 2) & K3;
      }
    }
#pragma unroll
    for (int v = 0; v < 3; ++v) {
      B[v][0] += Ne[v] & KF;         // fields 4k
      B[v][1] += (Ne[v] >> 4) & KF;  // fields 4k + 2
      B[v][2] += No[v] & KF;         // fields 4k + 1
      B[v][3] += (No[v] >> 4) & KF;  // fields 4k + 3
    }
  }
#pragma unroll
  for (int v = 0; v < 3; ++v)
#pragma unroll
    for (int w = 0; w < 4; ++w) xch[wave][4 * v + w][lane] = B[v][w];
  for (int o = 32; o; o >>= 1) seen += __shfl_xor(seen, o);
  if (lane == 0) seen_w[wave] = seen;
  __syncthreads();
  if (tid < 192) {  // word w = 4 v + q of all 256 lanes: 16 threads (one 16-lane group of a wave) per word
    const int w = tid >> 4, sub = tid & 15;
    uint32_t e = 0, o = 0;  // bytes 0, 2 / 1, 3 as 16-bit lanes
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int l = sub + 16 * i;
      const uint32_t x = xch[l >> 6][w][l & 63];
      e += x & 0x00FF00FFu;
      o += (x >> 8) & 0x00FF00FFu;
    }
#pragma unroll
    for (int s = 8; s; s >>= 1) {
      e += __shfl_xor(e, s);
      o += __shfl_xor(o, s);
    }
    if (sub == 0) {
      const int v = w >> 2, q = w & 3, off = q == 0 ? 0 : (q == 1 ? 2 : (q == 2 ? 1 : 3));
      cnt[off][v + 1] = e & 0xFFFFu;         // byte 0: field off
      cnt[4 + off][v + 1] = o & 0xFFFFu;     // byte 1: field 4 + off
      cnt[8 + off][v + 1] = e >> 16;         // byte 2
      cnt[12 + off][v + 1] = o >> 16;        // byte 3
    }
  }
  __syncthreads();
  if (tid < 128) {
    const int j = tid >> 2, v = tid & 3;
    uint32_t all = 0;
#pragma unroll
    for (int k = 0; k < WG / 64; ++k) all += seen_w[k];
    uint32_t t = 0;
    if (j < 16)
      t = v ? cnt[j][v] : all - cnt[j][1] - cnt[j][2] - cnt[j][3];
    else
      t = v ? 0u : all;  // (fields 16..31 are not output for L <= 16)
    part[(size_t)tid * gridDim.x + blockIdx.x] = t;
  }
}

// out[4 (L - 1 - j) + v] = the sum of the workgroups' partials of (j, v) (one workgroup per
// bin); bases p < L - 32 are all 0: n of value 0
__global__ __launch_bounds__(WG) void base_frequency_reduce_kernel(const unsigned long long* __restrict__ part,
                                                                   int parts, int64_t n, int L,
                                                                   unsigned long long* __restrict__ out) {
  const int b = blockIdx.x, j = b >> 2, v = b & 3;
  unsigned long long s = 0;
  for (int i = threadIdx.x; i < parts; i += WG) s += part[(size_t)b * parts + i];
#pragma unroll
  for (int o = 32; o; o >>= 1) s += __shfl_xor(s, o);
  __shared__ unsigned long long ws[WG / 64];
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < WG / 64; ++w) s += ws[w];
    if (j < 32 && j < L) out[4 * (L - 1 - j) + v] = s;
  }
  if (b == 0)
    for (int p = threadIdx.x; p < L - 32; p += WG)
      for (int k = 0; k < 4; ++k) out[4 * p + k] = k ? 0ull : (unsigned long long)n;
}

unsigned grid_for(int64_t n) {
  const int64_t b = sct::ceil_div(n, WG);
  return (unsigned)(b < 8192 ? (b > 0 ? b : 1) : 8192);
}

int words_for(int bits, int L) {
  const int64_t w = sct::ceil_div((int64_t)bits * L, 64);
  return (int)(w > 0 ? w : 1);
}

}  // namespace

extern "C" int sct_encode(int kind, const uint8_t* seqs, int64_t n, int64_t stride, int L,
                          uint64_t* codes, uint8_t* gc, uint8_t* flags, void* stream) {
  SCT_CHECK(kind == 2 || kind == 3, "kind must be 2 or 3");
  SCT_CHECK(n >= 0 && L >= 0 && stride >= L, "bad n/L/stride");
  SCT_CHECK(gc == nullptr || L <= 255, "gc output needs L <= 255");
  if (n == 0) return SCT_OK;
  SCT_CHECK(codes != nullptr && (L == 0 || seqs != nullptr), "NULL pointer");
  const int words = words_for(kind, L);
  constexpr int R = 4;  // tiled encoder: 4 x 256 records staged per iteration (28 KiB at L = 28)
  // (fewer records than one tile -- the drop-in's scalar calls -- skip the occupancy query)
  if (n >= R * WG && stride == L && words == 1 && L > 0 && L <= 64 && (uintptr_t)seqs % 16 == 0) {
    const size_t lds = (size_t)R * WG * L;
    const int64_t tiles = sct::ceil_div(n, R * WG);
    // one workgroup per tile (no loop), as a one-pass copy grid: 6.58 vs 7.68 ms for the
    // resident grid's loop on 100M 16-bp records (SCT_TUNE_ENCODE_GRID = 0 restores it)
    int64_t grid = tiles;
    if (sct::tune(SCT_TUNE_ENCODE_GRID, 1) != 1 || tiles >= (1LL << 31)) {
      sct::scalar_quiesce();
      // persistent: exactly the resident workgroups (a 4096 grid at 5 per CU left a partial
      // last round of workgroups, each looping over many tiles)
      int dev = 0, cus = 0, per_cu = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
      if (kind == 2)
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, encode_tiled_kernel<2, R>, WG, lds);
      else
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, encode_tiled_kernel<3, R>, WG, lds);
      grid = std::min<int64_t>(tiles, (int64_t)std::max(cus, 1) * std::max(per_cu, 1));
    }
    if (kind == 2)
      hipLaunchKernelGGL((encode_tiled_kernel<2, R>), dim3((unsigned)grid), dim3(WG), lds,
                         sct::as_stream(stream), seqs, n, L, codes, gc, flags);
    else
      hipLaunchKernelGGL((encode_tiled_kernel<3, R>), dim3((unsigned)grid), dim3(WG), lds,
                         sct::as_stream(stream), seqs, n, L, codes, gc, flags);
    SCT_LAUNCH_CHECK();
    return SCT_OK;
  }
  const bool dw = (L % 4 == 0) && (stride % 4 == 0) && ((uintptr_t)seqs % 4 == 0);
  hipLaunchKernelGGL(encode_kernel, dim3(grid_for(n)), dim3(WG), 0, sct::as_stream(stream), kind,
                     seqs, n, stride, L, words, dw, codes, gc, flags, (const int64_t*)nullptr,
                     (const int32_t*)nullptr);
  SCT_LAUNCH_CHECK();
  return SCT_OK;
}

extern "C" int sct_encode_var(int kind, const uint8_t* buf, const int64_t* starts, const int32_t* lens,
                              int64_t n, int words, uint64_t* codes, uint8_t* gc, uint8_t* flags, void* stream) {
  SCT_CHECK(kind == 2 || kind == 3, "kind must be 2 or 3");
  SCT_CHECK(n >= 0 && words >= 1, "bad n/words");
  if (n == 0) return SCT_OK;
  SCT_CHECK(buf && starts && lens && codes, "NULL pointer");
  if (words == 1) {
    hipLaunchKernelGGL(encode_var_kernel, dim3((unsigned)std::min<int64_t>(sct::ceil_div(n, WG), 1 << 30)), dim3(WG), 0, sct::as_stream(stream), kind, buf, n,
                       starts, lens, codes, gc, flags);
    SCT_LAUNCH_CHECK();
    return SCT_OK;
  }
  hipLaunchKernelGGL(encode_kernel, dim3(grid_for(n)), dim3(WG), 0, sct::as_stream(stream), kind, buf, n,
                     (int64_t)0, 0, words, false, codes, gc, flags, starts, lens);
  SCT_LAUNCH_CHECK();
  return SCT_OK;
}

extern "C" int sct_decode2(const uint64_t* codes, int64_t n, int words, int L, uint8_t* out,
                           void* stream) {
  SCT_CHECK(n >= 0 && words >= 1 && L >= 0, "bad n/words/L");
  if (n == 0 || L == 0) return SCT_OK;
  SCT_CHECK(codes && out, "NULL pointer");
  hipLaunchKernelGGL(decode2_kernel, dim3(grid_for(n)), dim3(WG), 0, sct::as_stream(stream), codes,
                     n, words, L, out);
  SCT_LAUNCH_CHECK();
  return SCT_OK;
}

extern "C" int sct_decode3(const uint64_t* codes, int64_t n, int words, int maxlen, uint8_t* out,
                           int32_t* lengths, int32_t* bad, void* stream) {
  SCT_CHECK(n >= 0 && words >= 1, "bad n/words");
  SCT_CHECK(maxlen >= (64 * words + 2) / 3, "maxlen %d < %d", maxlen, (64 * words + 2) / 3);
  if (n == 0) return SCT_OK;
  SCT_CHECK(codes && out && lengths && bad, "NULL pointer");
  hipLaunchKernelGGL(decode3_kernel, dim3(grid_for(n)), dim3(WG), 0, sct::as_stream(stream), codes,
                     n, words, maxlen, out, lengths, bad);
  SCT_LAUNCH_CHECK();
  return SCT_OK;
}

extern "C" int sct_gc_content(int kind, const uint64_t* codes, int64_t n, int words, int L,
                              int32_t* out, void* stream) {
  SCT_CHECK(kind == 2 || kind == 3, "kind must be 2 or 3");
  SCT_CHECK(n >= 0 && words >= 1 && L >= 0, "bad n/words/L");
  if (n == 0) return SCT_OK;
  SCT_CHECK(codes && out, "NULL pointer");
  hipLaunchKernelGGL(gc_kernel, dim3(grid_for(n)), dim3(WG), 0, sct::as_stream(stream), kind, codes,
                     n, words, L, out);
  SCT_LAUNCH_CHECK();
  return SCT_OK;
}

extern "C" int sct_hamming_pairs(int kind, const uint64_t* a, const uint64_t* b, int64_t n,
                                 int words, int32_t* out, void* stream) {
  SCT_CHECK(kind == 2 || kind == 3, "kind must be 2 or 3");
  SCT_CHECK(n >= 0 && words >= 1, "bad n/words");
  if (n == 0) return SCT_OK;
  SCT_CHECK(a && b && out, "NULL pointer");
  hipLaunchKernelGGL(hamming_kernel, dim3(grid_for(n)), dim3(WG), 0, sct::as_stream(stream), kind, a,
                     b, n, words, out);
  SCT_LAUNCH_CHECK();
  return SCT_OK;
}

extern "C" int sct_base_frequency(const uint64_t* codes, int64_t n, int L, uint64_t* out,
                                  void* stream) {
  SCT_CHECK(n >= 0 && L >= 0 && L <= 1024, "bad n/L");
  SCT_CHECK(out != nullptr && (n == 0 || codes != nullptr), "NULL pointer");
  if (L == 0) return SCT_OK;
  hipStream_t s = sct::as_stream(stream);
  if (n == 0) {
    SCT_HIP(hipMemsetAsync(out, 0, (size_t)L * 4 * 8, s));  // no code: every count 0
    return SCT_OK;
  }
  // 64-bit form: >= 32 codes per lane before the wave / workgroup reduction (at 8 per lane, 3.7M
  // codes on 1,024 workgroups, that epilogue -- 24 64-bit wave reductions per wave -- was most of
  // the kernel).  32-bit form (L <= 16): rounds of 15 codes per lane, never more than 255
  int blocks = (int)std::min<int64_t>(sct::ceil_div(n, 32 * WG), 512);
  if (L <= 16) {
    // one round per lane (15 codes) measured best: 3.69M codes 15.6-17.7 us, two rounds 13.2-21.4,
    // three 17.5-19.4, the 64-bit kernel 23.2-27.6 (profiles/ab_basefreq16_r05.jsonl)
    blocks = (int)std::max<int64_t>(std::min<int64_t>(sct::ceil_div(n, 15 * WG), 4096), sct::ceil_div(n, 255 * WG));
  }
  void* part = nullptr;
  SCT_HIP(sct::pool_alloc(&part, (size_t)128 * blocks * 8, s));
  if (L <= 16)
    hipLaunchKernelGGL(base_frequency16_kernel, dim3(blocks), dim3(WG), 0, s, codes, n, (unsigned long long*)part);
  else
    hipLaunchKernelGGL(base_frequency_kernel, dim3(blocks), dim3(WG), 0, s, codes, n, (unsigned long long*)part);
  hipError_t le = hipGetLastError();
  if (le == hipSuccess)
    hipLaunchKernelGGL(base_frequency_reduce_kernel, dim3(128), dim3(WG), 0, s, (const unsigned long long*)part,
                       blocks, n, L, reinterpret_cast<unsigned long long*>(out));
  if (le == hipSuccess) le = hipGetLastError();
  sct::pool_free(part, s);
  if (le != hipSuccess) return sct::fail(SCT_E_HIP, "kernel launch: %s", hipGetErrorString(le));
  return SCT_OK;
}

#define SCT_TRY(x)              \
  do {                          \
    int rc_ = (x);              \
    if (rc_ != SCT_OK) return rc_; \
  } while (0)
// ---------------------------------------------------------------- resident scalar server
// A scalar drop-in call (TwoBit.encode, hamming_distance, decode, gc_content: a batch of
// one) costs a kernel launch and its completion signal, ~15 us, while the work is a few
// hundred instructions.  Instead, the first such call of a host thread on a device launches
// one 64-lane server kernel that polls a page-locked, host-coherent mailbox over PCIe:
// the host writes the request (opcode, sizes, the packed inputs) and then its sequence
// number, all in one 64-B line the wave polls (larger payloads continue past it); the wave
// runs the same per-record device functions as the batch kernels (one record per lane,
// n <= 64) and answers with one checksummed 64-B response line (SrvMailbox::resp) that
// carries the sequence number, the status and small outputs.  The wave exits after
// idle_ticks of its wall clock without a
// request, on the mailbox's stop word, or never while a request is pending; it always
// writes its launch id to exit_gen last, so the host tells "exited" from "slow" without a
// HIP call, and relaunches (the pending request is served first) when it finds its
// request unanswered and the server gone.
namespace {
enum : uint32_t { OP_ENCODE = 1, OP_DECODE2 = 2, OP_DECODE3 = 3, OP_GC = 4, OP_HAMMING = 5 };
constexpr int kSrvIn = 1024, kSrvOut = 1024, kSrvMaxN = 64;

constexpr int kSrvInline = 28;  // payload bytes that ride in the request line itself
#ifndef SCT_SRV_COPIES
#define SCT_SRV_COPIES 4  // copies of the request line, one poll in flight on each
#endif
constexpr int kSrvCopies = SCT_SRV_COPIES;
static_assert(kSrvCopies >= 1 && kSrvCopies <= 8, "copies of the request line");

// One request line of 64 B: req[0] = seq (written last), req[1..7] = the packed fields,
// req[8..14] = the first 28 payload bytes, req[15] = line_check(req[0..14]); payload bytes
// 28.. follow in `more`.  The host writes the line kSrvCopies times (req, req_copy[..]) and the
// wave keeps one 64-B load in flight on each copy, so a scalar call (payload <= 28 B: a pair of
// one-limb codes, a 28-base record) is seen a fraction of a PCIe round trip after it lands
// (two loads in flight on the SAME line were slower than one: tools/scalar_floor_probe.hip).
// Nothing guarantees that the 16 dwords of one poll are one
// snapshot, so the wave takes a sequence number only when it is newer than the last served
// one (a copy not yet rewritten still shows the previous request) and the check word matches:
// a line mixing this request's seq with the previous request's fields is only polled again.
struct SrvMailbox {
  alignas(64) uint32_t req[16];
  uint32_t more[(kSrvIn - kSrvInline) / 4];
  // the other copies of the request line (dwords 0..15 of each row), 256 B apart
  alignas(256) uint32_t req_copy[kSrvCopies > 1 ? kSrvCopies - 1 : 1][64];
  // control (host)
  alignas(64) uint32_t stop;
  // response line (device), written by one 16-lane store: resp[0] = the served seq,
  // resp[1] = status, resp[2..14] = the outputs when they fit 52 bytes, resp[15] =
  // line_check(resp[0..14]).  No fence orders the line's dwords, so the host takes the line
  // only when the check matches (a torn write is waited out, never read).  Larger outputs go
  // to `out` first, behind a release fence.
  alignas(64) uint32_t resp[16];
  // the launch id on exit (device)
  alignas(64) uint32_t exit_gen;
  alignas(64) uint32_t out[kSrvOut / 4];
};
constexpr int kSrvInlineOut = 52;

// The check word of a 64-B line: the XOR of a hash of each of its first 15 dwords and their
// positions -- on the device one hash per lane and a 4-step XOR across the lanes of a DPP row,
// where a chained hash cost 15 dependent readlanes and multiplies on the request path (twice:
// request and response)
__host__ __device__ inline uint32_t word_mix(uint32_t w, uint32_t k) {
  uint32_t h = w ^ (0x9E3779B9u * (k + 1u));
  h ^= h >> 16;
  h *= 0x7FEB352Du;
  h ^= h >> 15;
  h *= 0x846CA68Bu;
  h ^= h >> 16;
  return h;
}
inline uint32_t line_check(const uint32_t* w) {
  uint32_t h = 0;
  for (uint32_t k = 0; k < 15; ++k) h ^= word_mix(w[k], k);
  return h;
}
// every lane: line_check of the 16-lane row holding it (lane r of the row holds dword r)
__device__ __forceinline__ uint32_t line_check_row(uint32_t v, int lane) {
  const int r = lane & 15;
  int h = (int)(r < 15 ? word_mix(v, (uint32_t)r) : 0u);
  h ^= __builtin_amdgcn_update_dpp(0, h, 0x128, 0xF, 0xF, false);  // row_ror:8
  h ^= __builtin_amdgcn_update_dpp(0, h, 0x124, 0xF, 0xF, false);  // row_ror:4
  h ^= __builtin_amdgcn_update_dpp(0, h, 0x122, 0xF, 0xF, false);  // row_ror:2
  h ^= __builtin_amdgcn_update_dpp(0, h, 0x121, 0xF, 0xF, false);  // row_ror:1
  return (uint32_t)h;
}
static_assert(offsetof(SrvMailbox, more) == 64, "the payload continues after the request line");

__device__ __forceinline__ uint32_t sys_load(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ int32_t sys_load(const int32_t* p) {
  return (int32_t)sys_load(reinterpret_cast<const uint32_t*>(p));
}

__global__ __launch_bounds__(64) void scalar_server_kernel(SrvMailbox* mb, uint32_t served, uint32_t gen,
                                                           uint64_t idle_ticks) {
  __shared__ uint8_t lut[2][256];
  __shared__ uint32_t in_l[kSrvIn / 4], out_l[kSrvOut / 4];
  const int lane = threadIdx.x;
  for (int c = lane; c < 256; c += 64) {
    lut[0][c] = lut_entry(2, c);
    lut[1][c] = lut_entry(3, c);
  }
  __syncthreads();
  // One poll in flight on each copy of the request line, and the wall clock read only every 32nd
  // round of polls (the idle exit).  Round-6 A/B of the library's C call (one TwoBit pair,
  // tools/scalar_floor_probe.hip, profiles/scalar_floor_r06/): two loads in flight on the same
  // line 4.81-4.84 us, one poll at a time 3.47-3.49 (the clock read on every poll +0.02-0.03),
  // one poll on each of two copies and the lane-parallel check word 2.09-2.22, on each of four
  // 1.98.  A polled mailbox answers in steps of its polls, so the time also depends on the host's
  // own time between calls: averaged over 0-2 us of it, 2.23-2.25 us with four copies, 2.5 with
  // two, 4.2 before round 6 (the polls bunched, see below).  Sleeping a calibrated quarter round
  // trip after every reload made it worse: 2.81-3.04.
  uint64_t t_last = wall_clock64();
  bool served_since = false;  // t_last is refreshed at the next clock read, off the request path
  // Serves the request `line` holds (lane r of each row holds dword r; a new seq, check word
  // matched).
  auto serve = [&](const uint32_t line) {
    const uint32_t seq = __builtin_amdgcn_readlane(line, 0);
    const uint32_t h1 = __builtin_amdgcn_readlane(line, 1), h2 = __builtin_amdgcn_readlane(line, 2),
                   h3 = __builtin_amdgcn_readlane(line, 3), h4 = __builtin_amdgcn_readlane(line, 4),
                   h5 = __builtin_amdgcn_readlane(line, 5), h6 = __builtin_amdgcn_readlane(line, 6),
                   h7 = __builtin_amdgcn_readlane(line, 7);
    auto off16 = [](uint32_t v) { return v == 0xFFFFu ? -1 : (int)v; };
    const uint32_t op = h1 & 0xFFu;
    const int kind = (int)((h1 >> 8) & 0xFFu), words = (int)(h1 >> 16);
    const int n = (int)(h2 & 0xFFFFu), L = (int)(h2 >> 16);
    const int stride = (int)(h3 & 0xFFFFu), maxlen = (int)(h3 >> 16);
    const int in_words = ((int)(h4 & 0xFFFFu) + 3) / 4, out_words = ((int)(h4 >> 16) + 3) / 4;
    const int io[2] = {off16(h5 & 0xFFFFu), off16(h5 >> 16)};
    const int oo[3] = {off16(h6 & 0xFFFFu), off16(h6 >> 16), off16(h7 & 0xFFFFu)};
    // payload: the first 7 dwords came with the line; the rest (if any) in one more round trip.
    // No acquire fence: the rest is read with system-scope loads (they bypass the caches) issued
    // only after this wave saw the sequence number the host stored after the payload, so they
    // return the new bytes; a system-scope acquire here was a whole-L2 invalidate
    // (buffer_inv sc0 sc1) on every request (round 6)
    if (lane >= 8 && lane < 15 && lane - 8 < in_words) in_l[lane - 8] = line;
    for (int k = kSrvInline / 4 + lane; k < in_words; k += 64) in_l[k] = sys_load(&mb->more[k - kSrvInline / 4]);
    for (int k = lane; k < out_words; k += 64) out_l[k] = 0u;
    __syncthreads();
    const uint8_t* in8 = reinterpret_cast<const uint8_t*>(in_l);
    uint8_t* out8 = reinterpret_cast<uint8_t*>(out_l);
    const int r = lane;
    if (r < n) {
      switch (op) {
        case OP_ENCODE: {
          RecordReader rd{in8 + io[0] + r * stride, false, 0u, -1};
          uint32_t g, fl;
          encode_record(lut[kind == 2 ? 0 : 1], kind, rd, L, words,
                        reinterpret_cast<uint64_t*>(out8 + oo[0]) + r * words, g, fl);
          if (oo[1] >= 0) out8[oo[1] + r] = (uint8_t)(g > 255 ? 255 : g);
          if (oo[2] >= 0) out8[oo[2] + r] = (uint8_t)fl;
          break;
        }
        case OP_DECODE2:
          decode2_record(reinterpret_cast<const uint64_t*>(in8 + io[0]) + r * words, words, L, out8 + oo[0] + r * L);
          break;
        case OP_DECODE3: {
          int32_t err;
          const int32_t len = decode3_record(reinterpret_cast<const uint64_t*>(in8 + io[0]) + r * words, words, maxlen,
                                             out8 + oo[0] + r * maxlen, err);
          reinterpret_cast<int32_t*>(out8 + oo[1])[r] = len;
          reinterpret_cast<int32_t*>(out8 + oo[2])[r] = err;
          break;
        }
        case OP_GC:
          reinterpret_cast<int32_t*>(out8 + oo[0])[r] =
              gc_record(kind, reinterpret_cast<const uint64_t*>(in8 + io[0]) + r * words, words, L);
          break;
        case OP_HAMMING:
          reinterpret_cast<int32_t*>(out8 + oo[0])[r] =
              hamming_record(kind, reinterpret_cast<const uint64_t*>(in8 + io[0]) + r * words,
                             reinterpret_cast<const uint64_t*>(in8 + io[1]) + r * words, words);
          break;
        default:
          break;
      }
    }
    __syncthreads();
    const bool inline_out = out_words * 4 <= kSrvInlineOut;
    if (!inline_out) {
      for (int k = lane; k < out_words; k += 64)
        __hip_atomic_store(&mb->out[k], out_l[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    }
    const uint32_t status = op >= OP_ENCODE && op <= OP_HAMMING ? 0u : 1u;
    uint32_t v = lane == 0 ? seq : lane == 1 ? status : (lane < 15 && inline_out && lane - 2 < out_words) ? out_l[lane - 2] : 0u;
    const uint32_t check = line_check_row(v, lane);
    if (lane == 15) v = check;
    if (lane < 16) __hip_atomic_store(&mb->resp[lane], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    served = seq;
    served_since = true;
  };
  // Every lane loads dword (lane & 15), so no lane branch surrounds the loads, and a copy's next
  // load is issued only after its line was examined (into the same register): the wait for the
  // oldest poll is then vmcnt(kSrvCopies - 1) and the other copies' loads stay in flight.  (An
  // array of copies in a loop over j was compiled with a full drain every round: the registers
  // rotated.)
  auto line_at = [&](int j) { return j == 0 ? mb->req + (lane & 15) : mb->req_copy[j - 1] + (lane & 15); };
  // The copies' polls are spread over a round trip: after the first poll and after every request
  // (when the polls in flight all came back while it was served) the next kSrvCopies - 1 polls are
  // issued a round trip / kSrvCopies apart (the round trip timed once here on the 100-MHz wall
  // clock); in between, each copy is reissued as soon as it was examined, which keeps the spacing.
  // Issued back to back instead, the polls stay bunched and a request waits for the next burst:
  // a saw-tooth of 2.0-2.9 us per C call over the host's own time between calls.
  uint64_t delta = 0, t_issue = 0;  // wall-clock ticks between spaced polls; the last one's issue
  int stagger = 0;                  // polls left to space
#ifndef SCT_SRV_NO_STAGGER
  {
    __builtin_amdgcn_s_waitcnt(0);
    const uint64_t t0 = wall_clock64();
    const uint32_t x = sys_load(line_at(0));
    __builtin_amdgcn_s_waitcnt(0);
    const uint64_t t1 = wall_clock64() + (__builtin_amdgcn_readlane(x, 0) & 0u);
    delta = min<uint64_t>((t1 - t0) / kSrvCopies, 100);
  }
#endif
  auto reload = [&](int j) {
    if (stagger > 0) {
      t_issue += delta;
      while (wall_clock64() < t_issue) {
      }
      --stagger;
    }
    return sys_load(line_at(j));
  };
  // (one load site per copy: with a second one on the request path the compiler gave the copies
  // new registers and moved them back at the end of every round, a full drain of the polls)
  auto step = [&](uint32_t& v, int j) {
    if ((int32_t)(__builtin_amdgcn_readlane(v, 0) - served) > 0 &&
        __builtin_amdgcn_readlane(line_check_row(v, lane), 0) == __builtin_amdgcn_readlane(v, 15)) {
      serve(v);
      t_issue = wall_clock64() - delta;  // this copy's poll goes out at once, the next ones spaced
      stagger = kSrvCopies;
    }
    v = reload(j);
  };
  static_assert(kSrvCopies == 2 || kSrvCopies == 4, "2 or 4 copies of the request line");
  t_issue = wall_clock64() - delta;
  stagger = kSrvCopies;
  uint32_t v0 = reload(0), v1 = reload(1);
  uint32_t v2 = kSrvCopies > 2 ? reload(2) : 0u, v3 = kSrvCopies > 2 ? reload(3) : 0u;
  for (uint32_t it = 1;; ++it) {
    step(v0, 0);
    step(v1, 1);
    if constexpr (kSrvCopies > 2) {
      step(v2, 2);
      step(v3, 3);
    }
    // the stop word costs a round trip of its own: looked at every 128th round of polls (~0.2 ms)
    if ((it & 127) == 0 && sys_load(&mb->stop) != 0u) break;
    if ((it & 31) == 0) {
      const uint64_t now = wall_clock64();
      if (served_since) t_last = now, served_since = false;
      else if (now - t_last > idle_ticks) break;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  if (lane == 0) __hip_atomic_store(&mb->exit_gen, gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

struct Server {
  int device = -1;
  SrvMailbox* mb = nullptr;      // host view
  SrvMailbox* mb_dev = nullptr;  // device view
  hipStream_t stream = nullptr;
  uint32_t seq = 0;
  std::atomic<uint32_t> gen{0};
  uint64_t idle_ticks = 0;
};

std::mutex g_srv_mu;
std::vector<Server*> g_servers;  // every server of the process (quiesce, exit)
std::atomic<int64_t> g_srv_launches{0};

template <class T>
T host_load(const T* p) {
  return __atomic_load_n(p, __ATOMIC_ACQUIRE);
}

bool server_running(const Server* sv) { return host_load(&sv->mb->exit_gen) != sv->gen.load(); }

// ask one server to exit and wait (bounded) for its exit mark; no HIP calls (process exit)
void server_stop(Server* sv, int64_t wait_us) {
  if (!server_running(sv)) return;
  __atomic_store_n(&sv->mb->stop, 1u, __ATOMIC_RELEASE);
  const auto t0 = std::chrono::steady_clock::now();
  while (server_running(sv) &&
         std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(wait_us)) {
  }
}

void stop_all_at_exit() {
  std::lock_guard<std::mutex> g(g_srv_mu);
  for (Server* sv : g_servers) server_stop(sv, 200000);
}

bool server_enabled() { return sct::tune(SCT_TUNE_SCALAR_SERVER, 1) != 0; }

// A host thread's servers (one per device).  When the thread ends its servers are stopped
// and their stream and mailbox freed, so thread churn does not pile up resident waves,
// streams and pinned memory; a server that does not confirm its exit is left alone (its
// mailbox must outlive it).
struct ThreadServers {
  Server* per_dev[64] = {};
  ~ThreadServers() {
    for (Server*& sv : per_dev) {
      if (!sv) continue;
      {  // out of the process list under the lock; the (bounded, up to 1 s) stop outside it
        std::lock_guard<std::mutex> g(g_srv_mu);
        g_servers.erase(std::remove(g_servers.begin(), g_servers.end(), sv), g_servers.end());
      }
      server_stop(sv, 1000000);
      if (server_running(sv)) {  // left alone, and back in the list for the exit-time stop
        std::lock_guard<std::mutex> g(g_srv_mu);
        g_servers.push_back(sv);
        continue;
      }
      int cur = -1;
      if (hipGetDevice(&cur) == hipSuccess && hipSetDevice(sv->device) == hipSuccess) {
        (void)hipStreamSynchronize(sv->stream);
        (void)hipStreamDestroy(sv->stream);
        (void)hipHostFree(sv->mb);
        (void)hipSetDevice(cur);
      }
      (void)hipGetLastError();
      delete sv;
      sv = nullptr;
    }
  }
};

// nullptr (error set) if the server cannot be created; callers then take the launch path
Server* server() {
  static thread_local ThreadServers mine;
  Server** per_dev = mine.per_dev;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  if (per_dev[dev]) return per_dev[dev];
  auto* sv = new Server();
  sv->device = dev;
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0) khz = 100000;
  const int64_t ms = sct::tune(SCT_TUNE_SCALAR_IDLE_MS, 5);
  sv->idle_ticks = (uint64_t)khz * (uint64_t)(ms > 0 ? ms : 5);
  if (hipStreamCreateWithFlags(&sv->stream, hipStreamNonBlocking) != hipSuccess ||
      hipHostMalloc((void**)&sv->mb, sizeof(SrvMailbox), hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess ||
      hipHostGetDevicePointer((void**)&sv->mb_dev, sv->mb, 0) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;  // leaked on this rare path; the launch path still works
  }
  memset(sv->mb, 0, sizeof(SrvMailbox));  // exit_gen == gen == 0: "not running"
  {
    std::lock_guard<std::mutex> g(g_srv_mu);
    if (g_servers.empty()) atexit(stop_all_at_exit);  // runs before HIP's own teardown
    g_servers.push_back(sv);
  }
  per_dev[dev] = sv;
  return sv;
}

int server_launch(Server* sv) {
  SCT_HIP(hipStreamSynchronize(sv->stream));  // the previous server has returned
  const uint32_t gen = sv->gen.load() + 1;
  __atomic_store_n(&sv->mb->stop, 0u, __ATOMIC_RELEASE);
  sv->gen.store(gen);
  hipLaunchKernelGGL(scalar_server_kernel, dim3(1), dim3(64), 0, sv->stream, sv->mb_dev, host_load(&sv->mb->resp[0]), gen,
                     sv->idle_ticks);
  SCT_LAUNCH_CHECK();
  g_srv_launches.fetch_add(1);
  return SCT_OK;
}

struct SrvIn {
  const void* p;
  size_t bytes;
};
struct SrvOut {
  void* p;
  size_t bytes;
};

// Returns SCT_OK when served, 1 when the request does not fit the server (the caller takes
// the launch path), or an error code.
template <int NI, int NO>
int srv_call(uint32_t op, int kind, int64_t n, int words, int L, int64_t stride, int maxlen, const SrvIn (&ins)[NI],
             const SrvOut (&outs)[NO]) {
  if (!server_enabled() || n > kSrvMaxN || stride > kSrvIn || L > kSrvOut || maxlen > kSrvOut || words > 255) return 1;
  // 8-byte aligned pieces (the widest element is a uint64 code): a pair of one-limb codes is 16 B
  // and rides in the request line; 16-byte alignment made it 32 B, past the 28 inline bytes, and
  // cost every hamming_distance call a second PCIe round trip for the rest (round 6)
  auto al = [](size_t x) { return (x + 7) & ~(size_t)7; };
  int32_t io[2] = {-1, -1}, oo[3] = {-1, -1, -1};
  size_t tin = 0, tout = 0;
  for (int k = 0; k < NI; ++k) {
    io[k] = (int32_t)tin;
    tin += al(ins[k].bytes);
  }
  for (int k = 0; k < NO; ++k) {
    if (!outs[k].p) continue;
    oo[k] = (int32_t)tout;
    tout += al(outs[k].bytes);
  }
  if (tin > (size_t)kSrvIn || tout > (size_t)kSrvOut) return 1;
  Server* sv = server();
  if (!sv) return 1;
  SrvMailbox* mb = sv->mb;
  uint32_t req[16] = {};  // the request line, written to both copies; seq last in each
  {  // payload bytes [0, 28) into req[8..14], the rest into `more`
    uint8_t pay[kSrvIn];
    for (int k = 0; k < NI; ++k)
      if (ins[k].bytes) memcpy(pay + io[k], ins[k].p, ins[k].bytes);
    memcpy(&req[8], pay, std::min<size_t>(tin, kSrvInline));
    if (tin > (size_t)kSrvInline) memcpy(mb->more, pay + kSrvInline, tin - kSrvInline);
  }
  auto o16 = [](int32_t v) { return v < 0 ? 0xFFFFu : (uint32_t)v; };
  req[1] = op | (uint32_t)kind << 8 | (uint32_t)words << 16;
  req[2] = (uint32_t)n | (uint32_t)L << 16;
  req[3] = (uint32_t)stride | (uint32_t)maxlen << 16;
  req[4] = (uint32_t)tin | (uint32_t)tout << 16;
  req[5] = o16(io[0]) | o16(io[1]) << 16;
  req[6] = o16(oo[0]) | o16(oo[1]) << 16;
  req[7] = o16(oo[2]);
  const uint32_t seq = ++sv->seq;
  req[0] = seq;
  req[15] = line_check(req);
  for (int j = 0; j < kSrvCopies; ++j) {
    uint32_t* line = j == 0 ? mb->req : mb->req_copy[j - 1];
    memcpy(line + 1, req + 1, 15 * 4);
    __atomic_store_n(&line[0], seq, __ATOMIC_RELEASE);
  }
  const auto t0 = std::chrono::steady_clock::now();
  uint32_t line[16];
  auto answered = [&]() {  // the whole response line of this request, check included
    if (host_load(&mb->resp[0]) != seq) return false;
    for (int k = 0; k < 16; ++k) line[k] = host_load(&mb->resp[k]);
    return line[0] == seq && line_check(line) == line[15];
  };
  for (uint32_t spin = 1;; ++spin) {
    if (answered()) break;
    if (!server_running(sv)) {
      if (answered()) break;  // served just before it left
      SCT_TRY(server_launch(sv));
      continue;
    }
    if ((spin & 4095) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10))
      return sct::fail(SCT_E_HIP, "scalar server: no answer in 10 s");
  }
  if (line[1] != 0) return sct::fail(SCT_E_HIP, "scalar server: bad request");
  const uint8_t* res = tout <= (size_t)kSrvInlineOut ? reinterpret_cast<const uint8_t*>(line + 2)
                                                     : reinterpret_cast<const uint8_t*>(mb->out);
  for (int k = 0; k < NO; ++k)
    if (outs[k].p && outs[k].bytes) memcpy(outs[k].p, res + oo[k], outs[k].bytes);
  return SCT_OK;
}
}  // namespace

namespace sct {
void scalar_quiesce() {
  std::lock_guard<std::mutex> g(g_srv_mu);
  for (Server* sv : g_servers) server_stop(sv, 1000000);
}
}  // namespace sct

extern "C" int sct_scalar_server_stop(void) {
  sct::scalar_quiesce();
  return SCT_OK;
}

extern "C" int sct_scalar_server_status(int64_t* launches, int* running) {
  if (launches) *launches = g_srv_launches.load();
  if (running) {
    std::lock_guard<std::mutex> g(g_srv_mu);
    int c = 0;
    for (Server* sv : g_servers) c += server_running(sv) ? 1 : 0;
    *running = c;
  }
  return SCT_OK;
}

// ---------------------------------------------------------------- host-pointer wrappers
// Every *_host call runs on the thread's host stage (sct::HostStage): small calls (the
// drop-in's scalar methods are batches of one) read their inputs from and write their
// outputs to the page-locked buffer directly (zero-copy: one launch and one stream sync,
// no allocation), larger ones pack inputs / outputs into one H2D and one D2H copy through
// the stage's device buffer, and only calls above kStageBytes allocate per call.
namespace {

struct In {
  const void* p;
  size_t bytes;
};
struct Out {
  void* p;
  size_t bytes;
};

// launch(ptrs, stream): ptrs = device-visible inputs then outputs (nullptr for a null host
// pointer).  zero_copy = false for kernels that update outputs atomically (PCIe atomics on
// host memory are not assumed).
template <int NI, int NO, class F>
int host_call(const In (&ins)[NI], const Out (&outs)[NO], bool zero_copy, F&& launch) {
  constexpr int N = NI + NO;
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  size_t off[N], total = 0;
  for (int k = 0; k < NI; ++k) {
    off[k] = total;
    total += al(ins[k].p ? ins[k].bytes : 0);
  }
  const size_t in_total = total;
  for (int k = 0; k < NO; ++k) {
    off[NI + k] = total;
    total += al(outs[k].p ? outs[k].bytes : 0);
  }
  sct::HostStage* st = sct::host_stage();
  if (!st) return SCT_E_HIP;
  void* ptr[N];
  if (zero_copy && total <= sct::kZeroCopyBytes) {
    SCT_TRY(sct::stage_reserve(st, total, 0));
    for (int k = 0; k < NI; ++k) {
      if (ins[k].p && ins[k].bytes) memcpy(st->pinned + off[k], ins[k].p, ins[k].bytes);
      ptr[k] = ins[k].p ? st->pinned_dev + off[k] : nullptr;
    }
    for (int k = 0; k < NO; ++k) ptr[NI + k] = outs[k].p ? st->pinned_dev + off[NI + k] : nullptr;
    SCT_TRY(launch(ptr, st->stream));
    // a few-microsecond kernel: poll instead of a blocking sync (saves the wake-up)
    hipError_t q;
    while ((q = hipStreamQuery(st->stream)) == hipErrorNotReady) {
    }
    SCT_HIP(q);
    for (int k = 0; k < NO; ++k)
      if (outs[k].p && outs[k].bytes) memcpy(outs[k].p, st->pinned + off[NI + k], outs[k].bytes);
    return SCT_OK;
  }
  if (total <= sct::kStageBytes) {
    SCT_TRY(sct::stage_reserve(st, total, total));
    for (int k = 0; k < NI; ++k) {
      if (ins[k].p && ins[k].bytes) memcpy(st->pinned + off[k], ins[k].p, ins[k].bytes);
      ptr[k] = ins[k].p ? st->dev + off[k] : nullptr;
    }
    for (int k = 0; k < NO; ++k) ptr[NI + k] = outs[k].p ? st->dev + off[NI + k] : nullptr;
    if (in_total) SCT_HIP(hipMemcpyAsync(st->dev, st->pinned, in_total, hipMemcpyHostToDevice, st->stream));
    SCT_TRY(launch(ptr, st->stream));
    if (total > in_total)
      SCT_HIP(hipMemcpyAsync(st->pinned + in_total, st->dev + in_total, total - in_total, hipMemcpyDeviceToHost,
                             st->stream));
    SCT_HIP(hipStreamSynchronize(st->stream));
    for (int k = 0; k < NO; ++k)
      if (outs[k].p && outs[k].bytes) memcpy(outs[k].p, st->pinned + off[NI + k], outs[k].bytes);
    return SCT_OK;
  }
  sct::DevBuf buf[N];
  for (int k = 0; k < NI; ++k) {
    ptr[k] = nullptr;
    if (!ins[k].p) continue;
    SCT_HIP(buf[k].alloc(ins[k].bytes));
    if (ins[k].bytes)
      SCT_HIP(hipMemcpyAsync(buf[k].p, ins[k].p, ins[k].bytes, hipMemcpyHostToDevice, st->stream));
    ptr[k] = buf[k].p;
  }
  for (int k = 0; k < NO; ++k) {
    ptr[NI + k] = nullptr;
    if (!outs[k].p) continue;
    SCT_HIP(buf[NI + k].alloc(outs[k].bytes));
    ptr[NI + k] = buf[NI + k].p;
  }
  SCT_TRY(launch(ptr, st->stream));
  for (int k = 0; k < NO; ++k)
    if (outs[k].p && outs[k].bytes)
      SCT_HIP(hipMemcpyAsync(outs[k].p, buf[NI + k].p, outs[k].bytes, hipMemcpyDeviceToHost, st->stream));
  SCT_HIP(hipStreamSynchronize(st->stream));
  return SCT_OK;
}
// Large element-wise calls (the *_array forms on host arrays): n items, item r of input k at
// ins[k].p + r * ins[k].bytes (bytes = PER ITEM here), likewise the outputs.  Chunks of items flow
// through NSTAGE device blocks on the thread's NSTAGE pipeline streams, so one chunk's H2D copy,
// another's kernel and a third's D2H copy overlap: the call runs at the PCIe rate of its larger
// direction.  Page-locked caller arrays (sct_host_pinned: the pool arrays the drop-in returns, torch
// pin_memory) are copied by DMA in place; pageable ones through the thread's pinned stage, filled
// and emptied by par_memcpy while the other stages' copies run.  launch(ptrs, m, stream) runs the
// kernel on m items at the device pointers.
constexpr size_t kStreamMinBytes = (size_t)8 << 20;  // below: one staged round trip (host_call)

template <int NI, int NO, class F>
int host_items(int64_t n, const In (&ins)[NI], const Out (&outs)[NO], F&& launch) {
  constexpr int NSTAGE = 3;
  size_t per = 0;
  for (int k = 0; k < NI; ++k) per += ins[k].bytes;
  for (int k = 0; k < NO; ++k) per += outs[k].p ? outs[k].bytes : 0;
  bool pin_in[NI > 0 ? NI : 1], pin_out[NO > 0 ? NO : 1];
  size_t stage_item = 0;  // pinned stage bytes per item (pageable arrays only)
  for (int k = 0; k < NI; ++k) {
    pin_in[k] = sct::host_range_pinned(ins[k].p, (size_t)n * ins[k].bytes);
    if (!pin_in[k]) stage_item += ins[k].bytes;
  }
  for (int k = 0; k < NO; ++k) {
    pin_out[k] = !outs[k].p || sct::host_range_pinned(outs[k].p, (size_t)n * outs[k].bytes);
    if (!pin_out[k]) stage_item += outs[k].bytes;
  }
  // ~16 MB of traffic per chunk, at least four chunks when there are enough items
  int64_t chunk = std::max<int64_t>(1 << 16, (int64_t)(((size_t)16 << 20) / std::max<size_t>(per, 1)));
  chunk = std::min<int64_t>(chunk, std::max<int64_t>(1 << 16, sct::ceil_div(n, 4)));
  chunk = std::min<int64_t>(chunk, n);
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  size_t doff[NI + NO], dtot = 0, hoff[NI + NO], htot = 0;
  for (int k = 0; k < NI + NO; ++k) {
    const size_t b = k < NI ? ins[k].bytes : (outs[k - NI].p ? outs[k - NI].bytes : 0);
    doff[k] = dtot;
    dtot += al((size_t)chunk * b);
    const bool staged = k < NI ? !pin_in[k] : !pin_out[k - NI];
    hoff[k] = htot;
    if (staged) htot += al((size_t)chunk * b);
  }
  sct::HostStage* hs = sct::host_stage();
  if (!hs) return SCT_E_HIP;
  if (htot) SCT_TRY(sct::stage_reserve(hs, NSTAGE * htot, 0));
  hipStream_t st[NSTAGE] = {};
  for (int k = 0; k < NSTAGE; ++k) {
    if (!hs->pipe[k]) SCT_HIP(hipStreamCreateWithFlags(&hs->pipe[k], hipStreamNonBlocking));
    st[k] = hs->pipe[k];
  }
  struct Streams {
    hipStream_t* s;
    ~Streams() {
      for (int k = 0; k < NSTAGE; ++k)
        if (s[k]) (void)hipStreamSynchronize(s[k]);
    }
  } guard{st};
  struct Blocks {
    void* p[NSTAGE] = {};
    hipStream_t* s;
    ~Blocks() {
      for (int k = 0; k < NSTAGE; ++k) sct::pool_free(p[k], s[k]);
    }
  } blk{{}, st};
  for (int k = 0; k < NSTAGE; ++k) SCT_HIP(sct::pool_alloc(&blk.p[k], dtot, st[k]));
  auto hstage = [&](int k, int a) { return hs->pinned + (size_t)k * htot + hoff[a]; };
  int64_t pend_r0[NSTAGE] = {}, pend_m[NSTAGE] = {};
  auto drain = [&](int k) -> int {
    if (pend_m[k] == 0) return SCT_OK;
    SCT_HIP(hipStreamSynchronize(st[k]));
    for (int o = 0; o < NO; ++o)
      if (outs[o].p && !pin_out[o])
        sct::par_memcpy(static_cast<uint8_t*>(outs[o].p) + (size_t)pend_r0[k] * outs[o].bytes, hstage(k, NI + o),
                        (size_t)pend_m[k] * outs[o].bytes);
    pend_m[k] = 0;
    return SCT_OK;
  };
  int64_t c = 0;
  for (int64_t r0 = 0; r0 < n; r0 += chunk, ++c) {
    const int k = (int)(c % NSTAGE);
    const int64_t m = std::min<int64_t>(chunk, n - r0);
    SCT_TRY(drain(k));  // (stage k's buffers are about to be reused)
    void* ptr[NI + NO];
    uint8_t* dev = static_cast<uint8_t*>(blk.p[k]);
    for (int a = 0; a < NI; ++a) {
      const uint8_t* src = static_cast<const uint8_t*>(ins[a].p) + (size_t)r0 * ins[a].bytes;
      const size_t b = (size_t)m * ins[a].bytes;
      if (!pin_in[a]) {
        sct::par_memcpy(hstage(k, a), src, b);
        src = hstage(k, a);
      }
      SCT_HIP(hipMemcpyAsync(dev + doff[a], src, b, hipMemcpyHostToDevice, st[k]));
      ptr[a] = dev + doff[a];
    }
    for (int o = 0; o < NO; ++o) ptr[NI + o] = outs[o].p ? dev + doff[NI + o] : nullptr;
    SCT_TRY(launch(ptr, m, st[k]));
    for (int o = 0; o < NO; ++o) {
      if (!outs[o].p) continue;
      uint8_t* dst = pin_out[o] ? static_cast<uint8_t*>(outs[o].p) + (size_t)r0 * outs[o].bytes : hstage(k, NI + o);
      SCT_HIP(hipMemcpyAsync(dst, dev + doff[NI + o], (size_t)m * outs[o].bytes, hipMemcpyDeviceToHost, st[k]));
    }
    pend_r0[k] = r0;
    pend_m[k] = m;
  }
  for (int k = 0; k < NSTAGE; ++k) SCT_TRY(drain(k));
  return SCT_OK;
}

// total bytes of an element-wise call
template <int NI, int NO>
size_t items_bytes(int64_t n, const In (&ins)[NI], const Out (&outs)[NO]) {
  size_t per = 0;
  for (int k = 0; k < NI; ++k) per += ins[k].bytes;
  for (int k = 0; k < NO; ++k) per += outs[k].p ? outs[k].bytes : 0;
  return (size_t)n * per;
}
}  // namespace

extern "C" int sct_encode_host(int kind, const uint8_t* seqs, int64_t n, int64_t stride, int L,
                               uint64_t* codes, uint8_t* gc, uint8_t* flags) {
  SCT_CHECK(kind == 2 || kind == 3, "kind must be 2 or 3");
  SCT_CHECK(n >= 0 && L >= 0 && stride >= L, "bad n/L/stride");
  if (n == 0) return SCT_OK;
  const int words = words_for(kind, L);
  const size_t in_bytes = (size_t)((n - 1) * stride + L);
  if (codes && (L == 0 || seqs) && (gc == nullptr || L <= 255)) {
    const int rc = srv_call<1, 3>(OP_ENCODE, kind, n, words, L, stride, 0, {{seqs, in_bytes}},
                                  {{codes, (size_t)n * words * 8}, {gc, (size_t)n}, {flags, (size_t)n}});
    if (rc != 1) return rc;
  }
  return host_call<1, 3>({{seqs, in_bytes}}, {{codes, (size_t)n * words * 8}, {gc, (size_t)n}, {flags, (size_t)n}},
                         true, [&](void** p, hipStream_t s) {
                           return sct_encode(kind, (const uint8_t*)p[0], n, stride, L, (uint64_t*)p[1], (uint8_t*)p[2],
                                             (uint8_t*)p[3], s);
                         });
}

extern "C" int sct_base_frequency_host(const uint64_t* codes, int64_t n, int L, uint64_t* out) {
  SCT_CHECK(n >= 0 && L >= 0 && L <= 1024, "bad n/L");
  if (L == 0) return SCT_OK;
  return host_call<1, 1>({{codes, (size_t)n * 8}}, {{out, (size_t)L * 4 * 8}}, false, [&](void** p, hipStream_t s) {
    return sct_base_frequency((const uint64_t*)p[0], n, L, (uint64_t*)p[1], s);
  });
}

// Host-resident stream (config 5): records live in host memory; chunks flow through
// NSTAGE device buffers on NSTAGE streams so that the H2D copy of one chunk, the encode
// of another and the D2H copy of a third overlap (PCIe-bound: L + 10 bytes per read cross
// the link).  Caller buffers the runtime already page-locks (hipHostMalloc, torch pin_memory, the
// caller's own hipHostRegister) are copied by DMA in place; pageable ones go through the thread's
// pinned stage, filled and emptied on the CPU while the other stages' copies and kernels run.  The
// library never page-locks caller memory itself (registering and unregistering ranges the runtime
// may also lock for its own pageable copies is not something to do behind the caller's back).
extern "C" int sct_encode_stream_host(int kind, const uint8_t* seqs, int64_t n, int L,
                                      uint64_t* codes, uint8_t* gc, uint8_t* flags,
                                      int64_t chunk) {
  SCT_CHECK(kind == 2 || kind == 3, "kind must be 2 or 3");
  SCT_CHECK(n >= 0 && L >= 1 && words_for(kind, L) == 1, "stream encode needs 1 <= L and one limb");
  SCT_CHECK(gc != nullptr && flags != nullptr && codes != nullptr && seqs != nullptr, "NULL pointer");
  if (n == 0) return SCT_OK;
  if (chunk <= 0) chunk = 1 << 24;
  constexpr int NSTAGE = 3;
  const bool pin_in = sct::host_range_pinned(seqs, (size_t)n * L);
  const bool pin_out = sct::host_range_pinned(codes, (size_t)n * 8) && sct::host_range_pinned(gc, (size_t)n) &&
                       sct::host_range_pinned(flags, (size_t)n);
  const bool staged = !pin_in || !pin_out;
  if (staged) chunk = std::min<int64_t>(chunk, 1 << 21);  // (a staged chunk: 2M reads, <= 2M * (L + 10) B)
  // at least four chunks when there are enough records, so the three stages overlap even for one
  // piece of a stream (a few million records)
  chunk = std::min<int64_t>(chunk, std::max<int64_t>(1 << 18, sct::ceil_div(n, 4)));
  chunk = std::min<int64_t>(chunk, n);
  const size_t in_b = pin_in ? 0 : (((size_t)chunk * L + 255) & ~(size_t)255);
  const size_t out_b = pin_out ? 0 : (size_t)chunk * 10;
  uint8_t* stage = nullptr;
  sct::HostStage* hs = sct::host_stage();
  if (!hs) return SCT_E_HIP;
  if (staged) {
    SCT_TRY(sct::stage_reserve(hs, NSTAGE * (in_b + out_b), 0));
    stage = hs->pinned;
  }
  static_assert(NSTAGE <= 3, "HostStage::pipe holds three streams");
  hipStream_t st[NSTAGE] = {};
  for (int k = 0; k < NSTAGE; ++k) {  // the thread's pipeline streams (kept across calls)
    if (!hs->pipe[k]) SCT_HIP(hipStreamCreateWithFlags(&hs->pipe[k], hipStreamNonBlocking));
    st[k] = hs->pipe[k];
  }
  struct Streams {
    hipStream_t* s;
    ~Streams() {  // (an early return leaves nothing in flight on the stage or the device buffers)
      for (int k = 0; k < NSTAGE; ++k)
        if (s[k]) (void)hipStreamSynchronize(s[k]);
    }
  } guard{st};
  // one device block per stage from the library's stream-ordered pool (records, then codes, GC,
  // flags), freed on its stage's stream before the streams go (declared after the guard)
  struct Blocks {
    void* p[NSTAGE] = {};
    hipStream_t* s;
    ~Blocks() {
      for (int k = 0; k < NSTAGE; ++k) sct::pool_free(p[k], s[k]);
    }
  } blk{{}, st};
  const size_t rec_b = ((size_t)chunk * L + 255) & ~(size_t)255;
  for (int k = 0; k < NSTAGE; ++k) SCT_HIP(sct::pool_alloc(&blk.p[k], rec_b + (size_t)chunk * 10, st[k]));
  struct StageDev {
    uint8_t* p;
  } din[NSTAGE], dcode[NSTAGE], dgc[NSTAGE], dfl[NSTAGE];
  for (int k = 0; k < NSTAGE; ++k) {
    uint8_t* b = static_cast<uint8_t*>(blk.p[k]);
    din[k].p = b;
    dcode[k].p = b + rec_b;
    dgc[k].p = b + rec_b + (size_t)chunk * 8;
    dfl[k].p = b + rec_b + (size_t)chunk * 9;
  }
  // stage k's pinned buffers: the input chunk, then codes / GC / flags of the chunk in flight
  auto h_in = [&](int k) { return stage + (size_t)k * (in_b + out_b); };
  auto h_out = [&](int k) { return stage + (size_t)k * (in_b + out_b) + in_b; };
  int64_t pend_r0[NSTAGE] = {}, pend_m[NSTAGE] = {};
  auto drain = [&](int k) -> int {  // wait for stage k's chunk; pageable outputs copied out
    if (pend_m[k] == 0) return SCT_OK;
    SCT_HIP(hipStreamSynchronize(st[k]));
    const int64_t r0 = pend_r0[k], m = pend_m[k];
    if (!pin_out) {
      memcpy(codes + r0, h_out(k), (size_t)m * 8);
      memcpy(gc + r0, h_out(k) + (size_t)chunk * 8, (size_t)m);
      memcpy(flags + r0, h_out(k) + (size_t)chunk * 9, (size_t)m);
    }
    pend_m[k] = 0;
    return SCT_OK;
  };
  int64_t c = 0;
  for (int64_t r0 = 0; r0 < n; r0 += chunk, ++c) {
    const int k = (int)(c % NSTAGE);  // stage k's previous chunk is ordered before on st[k]
    const int64_t m = std::min<int64_t>(chunk, n - r0);
    if (staged) SCT_TRY(drain(k));  // (its pinned buffers are about to be refilled)
    const uint8_t* src = seqs + r0 * L;
    if (!pin_in) {
      memcpy(h_in(k), src, (size_t)m * L);
      src = h_in(k);
    }
    SCT_HIP(hipMemcpyAsync(din[k].p, src, (size_t)m * L, hipMemcpyHostToDevice, st[k]));
    SCT_TRY(sct_encode(kind, (const uint8_t*)din[k].p, m, L, L, (uint64_t*)dcode[k].p, (uint8_t*)dgc[k].p,
                       (uint8_t*)dfl[k].p, st[k]));
    uint8_t* oc = pin_out ? reinterpret_cast<uint8_t*>(codes + r0) : h_out(k);
    uint8_t* og = pin_out ? gc + r0 : h_out(k) + (size_t)chunk * 8;
    uint8_t* of = pin_out ? flags + r0 : h_out(k) + (size_t)chunk * 9;
    SCT_HIP(hipMemcpyAsync(oc, dcode[k].p, (size_t)m * 8, hipMemcpyDeviceToHost, st[k]));
    SCT_HIP(hipMemcpyAsync(og, dgc[k].p, (size_t)m, hipMemcpyDeviceToHost, st[k]));
    SCT_HIP(hipMemcpyAsync(of, dfl[k].p, (size_t)m, hipMemcpyDeviceToHost, st[k]));
    pend_r0[k] = r0;
    pend_m[k] = m;
  }
  for (int k = 0; k < NSTAGE; ++k) SCT_TRY(drain(k));
  return SCT_OK;
}

extern "C" int sct_decode2_host(const uint64_t* codes, int64_t n, int words, int L, uint8_t* out) {
  SCT_CHECK(n >= 0 && words >= 1 && L >= 0, "bad n/words/L");
  if (n == 0 || L == 0) return SCT_OK;
  if (codes && out) {
    const int rc = srv_call<1, 1>(OP_DECODE2, 2, n, words, L, 0, 0, {{codes, (size_t)n * words * 8}}, {{out, (size_t)n * L}});
    if (rc != 1) return rc;
  }
  const In ii[1] = {{codes, (size_t)words * 8}};
  const Out oo[1] = {{out, (size_t)L}};
  if (codes && out && items_bytes(n, ii, oo) >= kStreamMinBytes)
    return host_items(n, ii, oo, [&](void** p, int64_t m, hipStream_t s) {
      return sct_decode2((const uint64_t*)p[0], m, words, L, (uint8_t*)p[1], s);
    });
  return host_call<1, 1>({{codes, (size_t)n * words * 8}}, {{out, (size_t)n * L}}, true,
                         [&](void** p, hipStream_t s) {
                           return sct_decode2((const uint64_t*)p[0], n, words, L, (uint8_t*)p[1], s);
                         });
}

extern "C" int sct_decode3_host(const uint64_t* codes, int64_t n, int words, int maxlen,
                                uint8_t* out, int32_t* lengths, int32_t* bad) {
  SCT_CHECK(n >= 0 && words >= 1, "bad n/words");
  if (n == 0) return SCT_OK;
  if (codes && out && lengths && bad && maxlen >= (64 * words + 2) / 3) {
    const int rc = srv_call<1, 3>(OP_DECODE3, 3, n, words, 0, 0, maxlen, {{codes, (size_t)n * words * 8}},
                                  {{out, (size_t)n * maxlen}, {lengths, (size_t)n * 4}, {bad, (size_t)n * 4}});
    if (rc != 1) return rc;
  }
  const In ii[1] = {{codes, (size_t)words * 8}};
  const Out oo[3] = {{out, (size_t)maxlen}, {lengths, 4}, {bad, 4}};
  if (codes && out && lengths && bad && items_bytes(n, ii, oo) >= kStreamMinBytes)
    return host_items(n, ii, oo, [&](void** p, int64_t m, hipStream_t s) {
      return sct_decode3((const uint64_t*)p[0], m, words, maxlen, (uint8_t*)p[1], (int32_t*)p[2], (int32_t*)p[3], s);
    });
  return host_call<1, 3>({{codes, (size_t)n * words * 8}},
                         {{out, (size_t)n * maxlen}, {lengths, (size_t)n * 4}, {bad, (size_t)n * 4}}, true,
                         [&](void** p, hipStream_t s) {
                           return sct_decode3((const uint64_t*)p[0], n, words, maxlen, (uint8_t*)p[1],
                                              (int32_t*)p[2], (int32_t*)p[3], s);
                         });
}

extern "C" int sct_gc_content_host(int kind, const uint64_t* codes, int64_t n, int words, int L,
                                   int32_t* out) {
  SCT_CHECK(n >= 0 && words >= 1, "bad n/words");
  if (n == 0) return SCT_OK;
  if ((kind == 2 || kind == 3) && L >= 0 && codes && out) {
    const int rc = srv_call<1, 1>(OP_GC, kind, n, words, L, 0, 0, {{codes, (size_t)n * words * 8}}, {{out, (size_t)n * 4}});
    if (rc != 1) return rc;
  }
  const In ii[1] = {{codes, (size_t)words * 8}};
  const Out oo[1] = {{out, 4}};
  if (codes && out && items_bytes(n, ii, oo) >= kStreamMinBytes)
    return host_items(n, ii, oo, [&](void** p, int64_t m, hipStream_t s) {
      return sct_gc_content(kind, (const uint64_t*)p[0], m, words, L, (int32_t*)p[1], s);
    });
  return host_call<1, 1>({{codes, (size_t)n * words * 8}}, {{out, (size_t)n * 4}}, true,
                         [&](void** p, hipStream_t s) {
                           return sct_gc_content(kind, (const uint64_t*)p[0], n, words, L, (int32_t*)p[1], s);
                         });
}

extern "C" int sct_hamming_pairs_host(int kind, const uint64_t* a, const uint64_t* b, int64_t n,
                                      int words, int32_t* out) {
  SCT_CHECK(n >= 0 && words >= 1, "bad n/words");
  if (n == 0) return SCT_OK;
  if ((kind == 2 || kind == 3) && a && b && out) {
    const int rc = srv_call<2, 1>(OP_HAMMING, kind, n, words, 0, 0, 0,
                                  {{a, (size_t)n * words * 8}, {b, (size_t)n * words * 8}}, {{out, (size_t)n * 4}});
    if (rc != 1) return rc;
  }
  const In ii[2] = {{a, (size_t)words * 8}, {b, (size_t)words * 8}};
  const Out oo[1] = {{out, 4}};
  if (a && b && out && items_bytes(n, ii, oo) >= kStreamMinBytes)
    return host_items(n, ii, oo, [&](void** p, int64_t m, hipStream_t s) {
      return sct_hamming_pairs(kind, (const uint64_t*)p[0], (const uint64_t*)p[1], m, words, (int32_t*)p[2], s);
    });
  return host_call<2, 1>({{a, (size_t)n * words * 8}, {b, (size_t)n * words * 8}}, {{out, (size_t)n * 4}}, true,
                         [&](void** p, hipStream_t s) {
                           return sct_hamming_pairs(kind, (const uint64_t*)p[0], (const uint64_t*)p[1], n, words,
                                                    (int32_t*)p[2], s);
                         });
}

