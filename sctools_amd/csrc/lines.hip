// Whitelist ingest on the device: Barcodes.from_whitelist (src/sctools/barcode.py:84-97)
// opens the file in binary mode, iterates its lines and TwoBit-encodes `line[:-1]` of each
// -- the LAST BYTE of every line is chopped, whatever it is (the '\n', or the last base of a
// file without a final newline; a CRLF line keeps its '\r', which then fails to encode).
//
// Lines of a binary file end at '\n' (the line includes it); a non-empty file whose last
// byte is not '\n' has one more line up to its end.  With P_g the position of line g's
// last byte ('\n', or the file's last byte), line g's chopped content is
// [P_{g-1} + 1, P_g): start = P_{g-1} + 1 (0 for g = 0), length = P_g - start.
//
// sct_whitelist_encode (the ingest Barcodes.from_whitelist takes, round 4): a count pass over
// 4 KiB tiles (16 bytes per thread, SWAR '\n' compares), a reduction of the tile counts, and an
// encode pass in which each line is encoded by the lane holding its end (below); no scan launch
// and no host synchronisation.
// sct_lines (kept for callers that want only the spans): two passes -- count each tile's line
// ends, exclusive-scan them, then store every end as the next line's start; the lengths follow
// from consecutive starts.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <atomic>

#include "sct_common.h"
#include "encode_common.h"
#include "tile_prefix.h"

namespace {

constexpr int WG = 256;
constexpr int TILE = WG * 16;

__device__ __forceinline__ uint32_t lf_mask(const uint8_t* __restrict__ buf, int64_t n, int64_t p0) {
  uint32_t m = 0;
  if (p0 + 16 <= n) {
    const uint4 v = *reinterpret_cast<const uint4*>(buf + p0);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t x = w[k] ^ 0x0A0A0A0Au;  // bit 7 of a byte set iff that byte is '\n'
      const uint32_t hi = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
      m |= (((hi >> 7) & 1u) | ((hi >> 14) & 2u) | ((hi >> 21) & 4u) | ((hi >> 28) & 8u)) << (4 * k);
    }
  } else {
    for (int j = 0; j < 16 && p0 + j < n; ++j) m |= (buf[p0 + j] == '\n' ? 1u : 0u) << j;
  }
  // the file's last byte ends a line too (a final line without '\n')
  if (n > 0 && p0 <= n - 1 && n - 1 < p0 + 16) m |= 1u << (n - 1 - p0);
  return m;
}

// the 16 bytes at p0 (zero past n) and their line ends (lf_mask)
__device__ __forceinline__ uint4 load16(const uint8_t* __restrict__ buf, int64_t n, int64_t p0) {
  if (p0 + 16 <= n) return *reinterpret_cast<const uint4*>(buf + p0);
  uint32_t w[4] = {0, 0, 0, 0};
  for (int j = 0; j < 16 && p0 + j < n; ++j) w[j >> 2] |= (uint32_t)buf[p0 + j] << (8 * (j & 3));
  return make_uint4(w[0], w[1], w[2], w[3]);
}
__device__ __forceinline__ uint32_t lf_mask_v(uint4 v, int64_t n, int64_t p0) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t m = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {  // (bytes past n are zero, never '\n')
    const uint32_t x = w[k] ^ 0x0A0A0A0Au;
    const uint32_t hi = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
    // bits 7, 15, 23, 31 -> 0..3 by one multiply: (hi >> 7) * (2^28 + 2^21 + 2^14 + 2^7) puts
    // byte j's bit at 28 + j and every other partial product at a distinct bit below 24 or
    // past 31 (tests/test_swar_host.py)
    m |= (((hi >> 7) * 0x10204080u) >> 28) << (4 * k);
  }
  if (n > 0 && p0 <= n - 1 && n - 1 < p0 + 16) m |= 1u << (n - 1 - p0);
  return m;
}

__global__ __launch_bounds__(WG) void line_count_kernel(const uint8_t* __restrict__ buf, int64_t n,
                                                        unsigned long long* __restrict__ counts) {
  const int64_t p0 = (int64_t)blockIdx.x * TILE + threadIdx.x * 16;
  const uint32_t c = p0 < n ? __popc(lf_mask(buf, n, p0)) : 0u;
  using BR = hipcub::BlockReduce<uint32_t, WG>;
  __shared__ typename BR::TempStorage tmp;
  const uint32_t tot = BR(tmp).Sum(c);
  if (threadIdx.x == 0) counts[blockIdx.x] = tot;
}

// line g ends at byte P_g, so line g + 1 starts at P_g + 1: every end found is stored as the
// next line's start (starts[0] = 0); the last line ends at the file's last byte
// (nlines = offsets[ntiles], read here: a capacity below it leaves the outputs untouched)
__global__ __launch_bounds__(WG) void line_starts_kernel(const uint8_t* __restrict__ buf, int64_t n,
                                                         const unsigned long long* __restrict__ offsets,
                                                         int64_t ntiles, int64_t cap, int64_t* __restrict__ starts) {
  const int64_t nlines = (int64_t)offsets[ntiles];
  if (nlines > cap) return;
  const int64_t p0 = (int64_t)blockIdx.x * TILE + threadIdx.x * 16;
  uint32_t m = p0 < n ? lf_mask(buf, n, p0) : 0u;
  using BS = hipcub::BlockScan<uint32_t, WG>;
  __shared__ typename BS::TempStorage tmp;
  uint32_t pre;
  BS(tmp).ExclusiveSum(__popc(m), pre);
  int64_t g = (int64_t)offsets[blockIdx.x] + pre;
  if (blockIdx.x == 0 && threadIdx.x == 0) starts[0] = 0;
  while (m) {
    const int j = __ffs(m) - 1;
    m &= m - 1;
    if (++g < nlines) starts[g] = p0 + j + 1;
  }
}

// chopped lengths: line g is [starts[g], P_g) with P_g = starts[g + 1] - 1 (the file's last
// byte for the last line); the longest by a workgroup maximum
__global__ __launch_bounds__(WG) void line_lens_kernel(const int64_t* __restrict__ starts,
                                                       const unsigned long long* __restrict__ total, int64_t cap,
                                                       int64_t nbytes, int32_t* __restrict__ lens,
                                                       int32_t* __restrict__ maxlen) {
  const int64_t nlines = (int64_t)*total;
  if (nlines > cap) return;  // workgroup-uniform: before the barrier below
  int32_t mx = 0;
  for (int64_t g = (int64_t)blockIdx.x * WG + threadIdx.x; g < nlines; g += (int64_t)gridDim.x * WG) {
    const int64_t end = g + 1 < nlines ? starts[g + 1] - 1 : nbytes - 1;
    const int32_t len = (int32_t)(end - starts[g]);
    lens[g] = len;
    mx = max(mx, len);
  }
#pragma unroll
  for (int s = 32; s; s >>= 1) mx = max(mx, __shfl_xor(mx, s));
  // same-address atomics serialise at L2 (8,192 of them cost ~0.1 ms): one per workgroup,
  // and only when it would raise the maximum already published
  __shared__ int32_t wmax[WG / 64];
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int w = 1; w < WG / 64; ++w) mx = max(mx, wmax[w]);
    if (mx > __hip_atomic_load(maxlen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(maxlen, mx);
  }
}

// ---------------------------------------------------------------- ingest in two passes (round 4)
// sct_whitelist_encode: wl_count_kernel counts each 16 KiB tile's line ends and its last one,
// tile_sums_reduce_kernel sums them into the 3-level tile sums (tile_prefix.h), and
// whitelist_fused_kernel reads the tiles again, takes its first tile's line number and the last
// line end before it from those sums, and encodes every line ending in its tiles: line g ends at
// the g-th line end P_g (a '\n', or the file's last byte) and its chopped content is
// [P_{g-1} + 1, P_g); each lane encodes the lines ending in its 16-byte pieces, the first one
// starting after the latest end before the piece.  The line count and the longest line stay on
// the device (no host synchronisation); a 62.7 MB whitelist's second read comes from the
// Infinity Cache.  A tile is NSUB = 4 sub-tiles of 4 KiB (the lane's piece j at 4096 j + 16 lane:
// every load instruction coalesced): 16 KiB per barrier pair and per wait for the loop's loads
// and stores, which drain at every wait (vmcnt(0): the stores' count varies by line).
constexpr int NSUB = 4, WTILE = NSUB * TILE;

// Fixed-stride files (every line S bytes with its '\n', the usual whitelist): the stride is the
// first line's length (S = its '\n' position + 1, taken from the file's first 64 bytes by every
// workgroup); a tile is flagged when any of its line ends is not at a position = S - 1 (mod S).
// The encode pass then numbers lines by arithmetic (line g ends at g S + S - 1) when no tile is
// flagged and S divides the file size.
constexpr int kMaxStride = 64;

// S, or 0 when the first 64 bytes hold no '\n'; every thread of the workgroup (one barrier)
__device__ __forceinline__ int file_stride(const uint8_t* __restrict__ buf, int64_t n, int* s_stride) {
  if (threadIdx.x == 0) {
    int S = 0;
    for (int k = 0; k < kMaxStride / 16 && !S; ++k) {
      const int64_t p = 16 * k;
      if (p >= n) break;
      const uint32_t m = lf_mask_v(load16(buf, n, p), n, p);  // (a file's last byte counts as an end)
      if (m) S = 16 * k + __ffs(m);
    }
    *s_stride = S;
  }
  __syncthreads();
  return *s_stride;
}

// spec_fail / spec_gen: when the one-read pass ran, it stored spec_gen in *spec_fail if the file is
// not its layout; any other value (the scratch word is not cleared: it may hold anything but
// this call's generation) means the one-read pass did it all and this pass returns at once.
// A grid of at most a few resident slots walks the tiles (a no-op launch then costs ~2 us less
// than one workgroup per tile).
__global__ __launch_bounds__(WG) void wl_count_kernel(const uint8_t* __restrict__ buf, int64_t n, int64_t ntiles,
                                                      sct::TileSums ts, int32_t* __restrict__ d_maxlen,
                                                      const unsigned* __restrict__ spec_fail, unsigned spec_gen) {
  if (spec_fail && *spec_fail != spec_gen) return;  // the one-read pass (whitelist_spec16_kernel) did it all
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    *d_maxlen = 0;  // (the encode pass raises it; no memset launch)
    *ts.fany = 0u;  // (the reduction ORs the tile flags into it)
  }
  __shared__ int s_stride;
  __shared__ uint32_t s_t0mod;
  __shared__ unsigned long long wc[WG / 64];
  __shared__ long long wl[WG / 64];
  __shared__ uint32_t wodd[WG / 64];
  const int S = file_stride(buf, n, &s_stride);
  const float invS = S ? 1.0f / (float)S : 0.0f;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t t0 = tile * WTILE;
    uint4 v[NSUB];
#pragma unroll
    for (int j = 0; j < NSUB; ++j) v[j] = load16(buf, n, t0 + j * TILE + threadIdx.x * 16);
    __syncthreads();  // (the previous tile's readers of the shared words are done)
    if (threadIdx.x == 0 && S) s_t0mod = (uint32_t)(t0 % S);
    __syncthreads();
    const uint32_t t0mod = S ? s_t0mod : 0u;
    unsigned long long c = 0;
    long long last = -1;
    uint32_t odd = S ? 0u : 1u;  // a line end off the stride
#pragma unroll
    for (int j = 0; j < NSUB; ++j) {
      const int64_t p0 = t0 + j * TILE + threadIdx.x * 16;
      const uint32_t m = p0 < n ? lf_mask_v(v[j], n, p0) : 0u;
      c += __popc(m);
      if (m) last = p0 + 31 - __clz(m);  // (sub-tiles in byte order)
      if (S && p0 < n) {
        // p0 mod S from the tile's t0 mod S and the in-tile offset r < 2^14 (float quotient: off by
        // at most one below, fixed by one compare)
        const uint32_t r = (uint32_t)(j * TILE + threadIdx.x * 16);
        const uint32_t q = (uint32_t)((float)r * invS);
        uint32_t ph = r - q * (uint32_t)S;
        if (ph >= (uint32_t)S) ph -= S;
        ph += t0mod;
        if (ph >= (uint32_t)S) ph -= S;
        uint32_t e = 0;  // the ends a stride-S file has in these bytes
        for (uint32_t b = (uint32_t)S - 1u - ph; b < 16u; b += (uint32_t)S) e |= 1u << b;
        const uint32_t valid = p0 + 16 <= n ? 0xFFFFu : (1u << (n - p0)) - 1u;
        odd |= (m ^ e) & valid;
      }
    }
#pragma unroll
    for (int o = 32; o; o >>= 1) {
      c += __shfl_xor(c, o);
      last = max(last, __shfl_xor(last, o));
    }
    const uint64_t oddw = __ballot(odd != 0u);
    if ((threadIdx.x & 63) == 0) {
      wc[threadIdx.x >> 6] = c;
      wl[threadIdx.x >> 6] = last;
      wodd[threadIdx.x >> 6] = oddw ? 1u : 0u;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t f = wodd[0];
      for (int w = 1; w < WG / 64; ++w) {
        c += wc[w];
        last = max(last, wl[w]);
        f |= wodd[w];
      }
      sct::tile_publish(ts, tile, c, last);
      ts.f0[tile] = f;
    }
  }
}

// one record of L <= 32 bytes at byte offset o (0..3) of an aligned dword window, one limb:
// dw(k) = dword k of the window (the window's dwords past the record's last are not read).
// Fast path, 4 bases per step without the LUT (VALU-bound before: the 32-step LUT loop cost
// ~380 instructions per line, PMC): an upper-case A/C/G/T byte c has TwoBit value
// v = x ^ (x >> 1), x = ((c >> 1) ^ (c >> 2)) & 3 (A 0, C 1, T 2, G 3), and a byte is one of
// them iff mapping v back through the table "ACTG" (one v_perm) returns it; the four values go
// MSB-first into 8 (TwoBit) or 12 (ThreeBit: v_perm through "2143") bits by two shift-ors.  Any
// other byte in the record (lower case, N, IUPAC, invalid) takes the LUT loop.
template <int KIND, class DW>
__device__ __forceinline__ void encode_line1(const uint8_t* lut, DW dw, int o, int L, uint64_t* out, uint32_t& g,
                                             uint32_t& fl) {
  constexpr uint64_t gcm = KIND == 2 ? 0x5555555555555555ull : 0x9249249249249249ull;
  uint64_t code = 0;
  uint32_t f = 0;
  if (L > 0) {
    const int last = (o + L - 1) >> 2;  // the window's last dword
    const int nfull = L >> 2, r = L & 3;
    uint32_t lo = dw(0), bad = 0;
    // whole dwords (4 bases each), then the last r bases
    for (int k = 0; k < nfull; ++k) {
      const uint32_t hi = dw(k + 1 <= last ? k + 1 : last);
      const uint32_t w = __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)o);  // bytes 4k .. 4k + 3
      lo = hi;
      const uint32_t x = ((w >> 1) ^ (w >> 2)) & 0x03030303u;
      const uint32_t v = x ^ ((x >> 1) & 0x01010101u);
      bad |= __builtin_amdgcn_perm(0u, 0x47544341u, v) ^ w;  // "ACTG"[v] == the byte?
      const uint32_t y = __builtin_amdgcn_perm(0u, KIND == 2 ? v : __builtin_amdgcn_perm(0u, 0x03040102u, v),
                                               0x00010203u);  // byte-reversed values
      if (KIND == 2) {  // v3 v2 at bits 0, 2 and v1 v0 at 16, 18; then v1 v0 down to 4, 6
        const uint32_t a = (y | (y >> 6)) & 0x000F000Fu;
        code = (code << 8) | ((a | (a >> 12)) & 0xFFu);
      } else {  // v3 v2 at bits 0, 3 and v1 v0 at 16, 19; then v1 v0 down to 6, 9
        const uint32_t a = (y | (y >> 5)) & 0x003F003Fu;
        code = (code << 12) | ((a | (a >> 10)) & 0xFFFu);
      }
    }
    if (r) {
      const uint32_t hi = dw(nfull + 1 <= last ? nfull + 1 : last);
      const uint32_t w = __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)o);
      const uint32_t x = ((w >> 1) ^ (w >> 2)) & 0x03030303u;
      const uint32_t v = x ^ ((x >> 1) & 0x01010101u);
      bad |= (__builtin_amdgcn_perm(0u, 0x47544341u, v) ^ w) & ((1u << (8 * r)) - 1u);
      const uint32_t y = __builtin_amdgcn_perm(0u, KIND == 2 ? v : __builtin_amdgcn_perm(0u, 0x03040102u, v),
                                               0x00010203u);
      uint32_t pk;
      if (KIND == 2) {
        const uint32_t a = (y | (y >> 6)) & 0x000F000Fu;
        pk = (a | (a >> 12)) & 0xFFu;
      } else {
        const uint32_t a = (y | (y >> 5)) & 0x003F003Fu;
        pk = (a | (a >> 10)) & 0xFFFu;
      }
      code = (code << (KIND * r)) | (pk >> (KIND * (4 - r)));
    }
    if (bad) {  // the LUT loop (ambiguous / invalid / lower-case bytes; rare: one read per byte)
      code = 0;
      for (int p = 0; p < L; ++p) {
        const uint32_t e = lut[(dw((o + p) >> 2) >> (8 * ((o + p) & 3))) & 0xFFu];
        code = (code << KIND) | (e & 7u);
        f |= e;
      }
    }
  }
  out[0] = code;
  g = (uint32_t)__popcll(code & gcm);
  fl = ((f & F_AMBIG) ? 1u : 0u) | ((f & F_INVALID) ? 2u : 0u);
}

// one record [rec, rec + L) of global memory through the LUT: the one-limb dword path of
// encode_var_kernel (encode.hip) for L <= 32, else the generic limb loop; too long for `words`
// limbs: flag 4
template <int KIND>
__device__ __forceinline__ void encode_line(const uint8_t* lut, const uint8_t* rec, int L, int words, uint64_t* out,
                                            uint32_t& g, uint32_t& fl) {
  if ((int64_t)KIND * L > 64 * (int64_t)words) {
    for (int w = 0; w < words; ++w) out[w] = 0;
    g = 0;
    fl = 4;
    return;
  }
  if (words == 1 && L <= 32) {
    const int o = (int)((uintptr_t)rec & 3);
    const uint32_t* dw = reinterpret_cast<const uint32_t*>(rec - o);
    encode_line1<KIND>(lut, [&](int k) { return dw[k]; }, o, L, out, g, fl);
    return;
  }
  RecordReader rd{rec, false, 0u, -1};
  encode_record(lut, KIND, rd, L, words, out, g, fl);
}

// A contiguous range of per_wg tiles per workgroup: the first tile's line number and last line
// end before it from the tile sums (once), then tile by tile (the next tile's bytes loaded while
// this one is worked), carrying both.  Within a tile the line ends are numbered without
// shuffle chains: a lane's exclusive count from ballots of its count's bits (mbcnt), the last
// end before its piece from the nearest lower lane with one (one bpermute), the wave's totals
// by readlane; the 4 sub-tiles x 4 waves then combine through LDS.  The tile's bytes are staged
// in LDS and every line that starts inside the tile is encoded from there (ds_read; only a
// tile's first line may start before it).
template <int KIND>
__global__ __launch_bounds__(WG) void whitelist_fused_kernel(
    const uint8_t* __restrict__ buf, int64_t n, int64_t ntiles, int64_t per_wg, sct::TileSums ts, int direct,
    int64_t cap, int words, uint64_t* __restrict__ codes, int64_t* __restrict__ starts, int32_t* __restrict__ lens,
    uint8_t* __restrict__ gc, uint8_t* __restrict__ flags, unsigned long long* __restrict__ d_nlines,
    int32_t* __restrict__ d_maxlen, const unsigned* __restrict__ spec_fail, unsigned spec_gen) {
  if (spec_fail && *spec_fail != spec_gen) return;  // the one-read pass did it all
  __shared__ uint8_t lut[256];
  __shared__ uint4 tile_bytes[WTILE / 16 + 1];  // (+16: encode_line1's dword reads stay inside)
  __shared__ uint32_t w_cnt[NSUB][WG / 64];
  __shared__ int32_t w_last[NSUB][WG / 64];  // in-tile offset of the wave's last line end, -1: none
  __shared__ unsigned long long s_excl;
  __shared__ long long s_excl_last;
  __shared__ unsigned long long red[3][WG / 64];
  __shared__ int32_t w_max[WG / 64];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  int64_t tile = (int64_t)blockIdx.x * per_wg;
  if (tile >= ntiles) return;  // (the whole workgroup)
  const int64_t tend = tile + per_wg < ntiles ? tile + per_wg : ntiles;
  for (int c = t; c < 256; c += WG) lut[c] = lut_entry(KIND, c);
  if (t == 0) tile_bytes[WTILE / 16] = make_uint4(0, 0, 0, 0);
  uint4 cur[NSUB];
#pragma unroll
  for (int j = 0; j < NSUB; ++j) cur[j] = load16(buf, n, tile * WTILE + j * TILE + t * 16);
  lds_u32* lds32 = as_lds32(tile_bytes);
  __shared__ int s_stride;
  __shared__ uint32_t s_fany;
  const int S = file_stride(buf, n, &s_stride);  // (its barrier also covers the LUT)
  // direct: the tile prefix and the flags straight from the per-tile words (no reduction launch)
  if (direct) sct::tile_prefix_direct<WG>(ts, tile, ntiles, &s_excl, &s_excl_last, &s_fany, red);
  const uint32_t fany = direct ? s_fany : *ts.fany;
  if (S > 0 && fany == 0u && n % S == 0 && words == 1 && KIND * (S - 1) <= 64) {
    // a fixed-stride file: line g is [g S, g S + S - 1); the lines ending in a tile are
    // g in [t0 / S, t1 / S), one per thread (consecutive lanes, consecutive lines: every store
    // coalesced), no numbering
    const int L = S - 1;
    if (L == 16) {
      // 16-base lines (10x whitelists): each thread takes lines of the workgroup's whole range
      // straight from memory (L2 / the Infinity Cache: the count pass just read them) -- 4 or 5
      // aligned dwords per line, all loads issued at once, no LDS staging, no barriers
      const int64_t t1 = tend * WTILE < n ? tend * WTILE : n, gB = t1 / S;
      const int64_t gend = gB < cap ? gB : (cap > 0 ? cap : 0);
      constexpr int U = 4;  // lines per thread per step, all their loads issued before any is used
      for (int64_t g0 = tile * WTILE / S + t; g0 < gend; g0 += U * WG) {
        uint32_t d[U][5];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int64_t g = g0 + (int64_t)u * WG, start = g * S;
          const uint32_t o = (uint32_t)(start & 3);
          if (g < gend && start - o + 20 <= n) {
            const uint32_t* w = reinterpret_cast<const uint32_t*>(buf + (start - o));
#pragma unroll
            for (int k = 0; k < 4; ++k) d[u][k] = w[k];
            d[u][4] = o ? w[4] : 0u;
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int64_t g = g0 + (int64_t)u * WG, start = g * S;
          if (g >= gend) break;
          const uint32_t o = (uint32_t)(start & 3);
          uint32_t gg, fl;
          bool done = false;
          if (start - o + 20 <= n) {
            uint64_t code = 0;
            uint32_t bad = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const uint32_t x = __builtin_amdgcn_alignbyte(d[u][k + 1], d[u][k], o);
              const uint32_t uu = ((x >> 1) ^ (x >> 2)) & 0x03030303u;
              const uint32_t v = uu ^ ((uu >> 1) & 0x01010101u);
              bad |= __builtin_amdgcn_perm(0u, 0x47544341u, v) ^ x;
              const uint32_t y =
                  __builtin_amdgcn_perm(0u, KIND == 2 ? v : __builtin_amdgcn_perm(0u, 0x03040102u, v), 0x00010203u);
              if (KIND == 2) {
                const uint32_t a = (y | (y >> 6)) & 0x000F000Fu;
                code = (code << 8) | ((a | (a >> 12)) & 0xFFu);
              } else {
                const uint32_t a = (y | (y >> 5)) & 0x003F003Fu;
                code = (code << 12) | ((a | (a >> 10)) & 0xFFFu);
              }
            }
            if (!bad) {
              codes[g] = code;
              gg = (uint32_t)__popcll(code & (KIND == 2 ? 0x5555555555555555ull : 0x9249249249249249ull));
              fl = 0;
              done = true;
            }
          }
          // a line with another byte (the LUT), or the file's last line (its window would read
          // past the buffer)
          if (!done) encode_line<KIND>(lut, buf + start, L, 1, codes + g, gg, fl);
          starts[g] = start;
          lens[g] = L;
          if (gc) gc[g] = (uint8_t)gg;
          if (flags) flags[g] = (uint8_t)fl;
        }
      }
      tile = tend;  // (the range is done)
    }
    for (; tile < tend; ++tile) {
      const int64_t t0 = tile * WTILE, t1 = t0 + WTILE < n ? t0 + WTILE : n;
      __syncthreads();  // the previous tile's readers of tile_bytes are done
#pragma unroll
      for (int j = 0; j < NSUB; ++j) tile_bytes[j * WG + t] = cur[j];
      if (tile + 1 < tend) {
#pragma unroll
        for (int j = 0; j < NSUB; ++j) cur[j] = load16(buf, n, t0 + WTILE + j * TILE + t * 16);
      }
      __syncthreads();
      const int64_t gB = t1 / S;
      for (int64_t g = t0 / S + t; g < gB; g += WG) {
        if (g >= cap) break;
        const int64_t start = g * S;
        uint32_t gg, fl;
        if (start >= t0) {
          const int off = (int)(start - t0), o = off & 3, w0 = off >> 2;
          encode_line1<KIND>(lut, [&](int k) { return lds32[w0 + k]; }, o, L, codes + g, gg, fl);
        } else {
          encode_line<KIND>(lut, buf + start, L, 1, codes + g, gg, fl);
        }
        starts[g] = start;
        lens[g] = L;
        if (gc) gc[g] = (uint8_t)(gg > 255 ? 255 : gg);
        if (flags) flags[g] = (uint8_t)fl;
      }
    }
    if (t == 0) {
      if (L > __hip_atomic_load(d_maxlen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(d_maxlen, L);
      if (tend == ntiles) *d_nlines = (unsigned long long)(n / S);
    }
    return;
  }
  if (!direct) sct::tile_prefix<WG>(ts, tile, &s_excl, &s_excl_last, red);
  uint64_t g_base = s_excl;
  long long last_base = s_excl_last;
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  int32_t mx = 0;
  for (; tile < tend; ++tile) {
    const int64_t t0 = tile * WTILE;
    const bool more = tile + 1 < tend;
    uint4 nxt[NSUB];
#pragma unroll
    for (int j = 0; j < NSUB; ++j)
      nxt[j] = more ? load16(buf, n, t0 + WTILE + j * TILE + t * 16) : make_uint4(0, 0, 0, 0);
    uint32_t m[NSUB], xc[NSUB];
    int32_t xl[NSUB];
    __syncthreads();  // the previous tile's readers of tile_bytes / w_cnt / w_last are done
#pragma unroll
    for (int j = 0; j < NSUB; ++j) {
      const int64_t p0 = t0 + j * TILE + t * 16;
      m[j] = p0 < n ? lf_mask_v(cur[j], n, p0) : 0u;
      tile_bytes[j * WG + t] = cur[j];
      cur[j] = nxt[j];

      const uint32_t c = __popc(m[j]);  // <= 16: five bits
      uint32_t ex = 0, tot = 0;
#pragma unroll
      for (int b = 0; b < 5; ++b) {
        const uint64_t bb = __ballot((c >> b) & 1u);
        ex += (uint32_t)__popcll(bb & lt_mask) << b;
        tot += (uint32_t)__popcll(bb) << b;
      }
      xc[j] = ex;
      const int32_t mylast = m[j] ? j * TILE + t * 16 + 31 - __clz(m[j]) : -1;
      const uint64_t has = __ballot(m[j] != 0u), lower = has & lt_mask;
      const int src = lower ? 63 - __clzll(lower) : lane;
      const int32_t pl = __shfl(mylast, src);
      xl[j] = lower ? pl : -1;
      if (lane == 0) {
        w_cnt[j][wave] = tot;
        w_last[j][wave] = has ? __builtin_amdgcn_readlane(mylast, 63 - __clzll(has)) : -1;
      }
    }
    __syncthreads();
    // the tile's outputs from its first line on (uniform bases), and how many of them fit
    const uint32_t cap_rel = (int64_t)g_base >= cap ? 0u
                             : (uint32_t)(cap - (int64_t)g_base < (int64_t)0xFFFFFFFF ? cap - (int64_t)g_base : 0xFFFFFFFF);
    uint64_t* codes_t = codes + g_base * (uint64_t)words;
    int64_t* starts_t = starts + g_base;
    int32_t* lens_t = lens + g_base;
    uint8_t* gc_t = gc ? gc + g_base : nullptr;
    uint8_t* flags_t = flags ? flags + g_base : nullptr;
    // prefix of the (sub-tile, wave) pieces before this one, in byte order; the tile's totals
    uint32_t pre = 0, tot = 0;
    int32_t plast = -1, tlast = -1;
#pragma unroll
    for (int j = 0; j < NSUB; ++j)
#pragma unroll
      for (int w = 0; w < WG / 64; ++w) {
        const uint32_t cw = w_cnt[j][w];
        const int32_t lw = w_last[j][w];
        tot += cw;
        tlast = max(tlast, lw);
      }
#pragma unroll
    for (int j = 0; j < NSUB; ++j) {
      uint32_t pj = pre;
      int32_t lj = plast;
#pragma unroll
      for (int w = 0; w < WG / 64; ++w)
        if (w < wave) {
          pj += w_cnt[j][w];
          lj = max(lj, w_last[j][w]);
        }
      uint32_t mm = m[j];
      const int32_t prev_in = max(lj, xl[j]);  // in-tile offset of the last end before the piece, -1: none
      // in-tile offsets and line numbers relative to the tile's first line (32-bit: the stores
      // take a uniform base + a 32-bit offset, no 64-bit address arithmetic per line)
      const int32_t p0r = j * TILE + t * 16;
      int64_t prev = prev_in >= 0 ? t0 + prev_in : last_base;  // global position of the previous end
      for (uint32_t li = pj + xc[j]; mm; ++li) {
        const int b = __ffs(mm) - 1;
        mm &= mm - 1;
        const int32_t Pr = p0r + b;
        const int64_t start = prev + 1;
        const int32_t L = (int32_t)(t0 + Pr - start);
        prev = t0 + Pr;
        mx = max(mx, L);
        if (li < cap_rel) {
          uint32_t gg, fl;
          if (start >= t0 && words == 1 && KIND * L <= 64) {  // inside the tile: from its LDS copy
            const int off = (int)(start - t0), o = off & 3, w0 = off >> 2;
            encode_line1<KIND>(lut, [&](int k) { return lds32[w0 + k]; }, o, L, codes_t + li, gg, fl);
          } else {
            encode_line<KIND>(lut, buf + start, L, words, codes_t + (size_t)li * words, gg, fl);
          }
          starts_t[li] = start;
          lens_t[li] = L;
          if (gc) gc_t[li] = (uint8_t)(gg > 255 ? 255 : gg);
          if (flags) flags_t[li] = (uint8_t)fl;
        }
      }
      // the next sub-tile's pieces follow all of this one's
#pragma unroll
      for (int w = 0; w < WG / 64; ++w) {
        pre += w_cnt[j][w];
        plast = max(plast, w_last[j][w]);
      }
    }
    g_base += tot;
    if (tlast >= 0) last_base = t0 + tlast;
  }
#pragma unroll
  for (int s = 32; s; s >>= 1) mx = max(mx, __shfl_xor(mx, s));
  if (lane == 0) w_max[wave] = mx;
  __syncthreads();
  if (t == 0) {
#pragma unroll
    for (int w = 1; w < WG / 64; ++w) mx = max(mx, w_max[w]);
    if (mx > __hip_atomic_load(d_maxlen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(d_maxlen, mx);
    if (tend == ntiles) *d_nlines = g_base;
  }
}

// persistent grid: the resident workgroup slots of `kernel` (at most ntiles)
int64_t resident_slots(const void* kernel, int64_t ntiles) {
  sct::scalar_quiesce();
  int dev = 0, cus = 256, per_cu = 0;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, WG, 0) != hipSuccess || per_cu <= 0) per_cu = 4;
  return std::max<int64_t>(1, std::min<int64_t>(ntiles, (int64_t)cus * per_cu));
}

// Scratch of one call, allocated and freed in stream order from the library's private memory
// pool (sct::pool_alloc: its memory stays in the pool, so repeated calls map nothing).
struct StreamBuf {
  void* p = nullptr;
  hipStream_t s = nullptr;
  ~StreamBuf() {
    sct::pool_free(p, s);
  }
  hipError_t alloc(size_t bytes, hipStream_t st) {
    s = st;
    return sct::pool_alloc(&p, bytes, st);
  }
};

}  // namespace

// Lines of a device buffer (binary mode) with the [:-1] chop: starts / lens of nlines lines
// (capacity max_lines; a sizing call with max_lines < the count fills nothing), the longest
// chopped length in *max_len.  Synchronous on `stream` (one synchronisation).
extern "C" int sct_lines(const uint8_t* d_buf, int64_t nbytes, int64_t max_lines, int64_t* d_starts,
                         int32_t* d_lens, int64_t* nlines, int32_t* max_len, void* stream) {
  SCT_CHECK(nlines != nullptr && max_len != nullptr, "NULL pointer");
  SCT_CHECK(nbytes >= 0 && (nbytes == 0 || d_buf != nullptr), "bad buffer");
  *nlines = 0;
  *max_len = 0;
  if (nbytes == 0) return SCT_OK;
  hipStream_t s = sct::as_stream(stream);
  const int64_t ntiles = sct::ceil_div(nbytes, TILE);
  // line_count_kernel: one workgroup per tile, < 2^32 threads per launch
  SCT_CHECK(ntiles * WG < (1LL << 32), "buffer too large: %lld bytes (one launch covers < %lld)", (long long)nbytes,
            (long long)(((1LL << 32) / WG) * TILE));
  size_t tb = 0;
  SCT_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, (unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                           (int)(ntiles + 1), s));
  // one scratch block: tile counts, their offsets, the scan's temporary storage, the maximum
  const size_t cb = (size_t)(ntiles + 1) * 8, tb_al = (tb + 255) & ~(size_t)255;
  StreamBuf scratch;
  SCT_HIP(scratch.alloc(2 * cb + tb_al + 8, s));
  unsigned long long* cnt = (unsigned long long*)scratch.p;
  unsigned long long* off = cnt + (ntiles + 1);
  void* tmp = (uint8_t*)scratch.p + 2 * cb;
  int32_t* mx = (int32_t*)((uint8_t*)tmp + tb_al);
  SCT_HIP(hipMemsetAsync(cnt, 0, cb, s));
  hipLaunchKernelGGL(line_count_kernel, dim3((unsigned)ntiles), dim3(WG), 0, s, d_buf, nbytes, cnt);
  SCT_LAUNCH_CHECK();
  SCT_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tb, cnt, off, (int)(ntiles + 1), s));
  const unsigned long long* d_total = off + ntiles;
  unsigned long long total = 0;
  if (max_lines <= 0 || !d_starts || !d_lens) {  // a sizing call: the count only
    SCT_HIP(hipMemcpyAsync(&total, d_total, 8, hipMemcpyDeviceToHost, s));
    SCT_HIP(hipStreamSynchronize(s));
    *nlines = (int64_t)total;
    return SCT_OK;
  }
  // the spans follow without waiting for the count: the kernels read it on the device and
  // leave the outputs untouched when it exceeds max_lines; one synchronisation at the end
  hipLaunchKernelGGL(line_starts_kernel, dim3((unsigned)ntiles), dim3(WG), 0, s, d_buf, nbytes,
                     (const unsigned long long*)off, ntiles, max_lines, d_starts);
  SCT_LAUNCH_CHECK();
  SCT_HIP(hipMemsetAsync(mx, 0, 4, s));
  hipLaunchKernelGGL(line_lens_kernel, dim3((unsigned)std::min<int64_t>(sct::ceil_div(max_lines, WG), 2048)),
                     dim3(WG), 0, s, (const int64_t*)d_starts, d_total, max_lines, nbytes, d_lens, mx);
  SCT_LAUNCH_CHECK();
  int32_t mlen = 0;
  SCT_HIP(hipMemcpyAsync(&total, d_total, 8, hipMemcpyDeviceToHost, s));
  SCT_HIP(hipMemcpyAsync(&mlen, mx, 4, hipMemcpyDeviceToHost, s));
  SCT_HIP(hipStreamSynchronize(s));
  *nlines = (int64_t)total;
  *max_len = (int64_t)total <= max_lines ? mlen : 0;
  return SCT_OK;
}

// One pass: lines + [:-1] chop + encode (whitelist_fused_kernel), asynchronous on `stream`: the
// line count and the longest chopped line go to d_nlines / d_maxlen; lines g < max_lines are
// written (starts, lens, words limbs of codes, gc and flags nullable; flags bit 2 = a line
// too long for `words` limbs).
// One read of a 10x-style whitelist: the file is ASSUMED to be lines of 16 bases
// and a '\n' (stride 17, the size a multiple of 17) -- line g is [17 g, 17 g + 16) -- and every
// line is encoded straight from memory as the fixed-stride branch of whitelist_fused_kernel does,
// while the assumption is CHECKED on the same bytes: the stride taken from the file's first line
// must be 17, byte 17 g + 16 must be a '\n', and no line's 16 bytes may hold one (an A/C/G/T line
// holds none; a line through the LUT path is searched).  Any failure stores this call's generation
// `gen` in *fail, and the count and encode passes that follow in the stream (which return at once
// unless *fail holds gen -- the word is never cleared, so no memset launch precedes the pass: a
// stale value can only be another call's generation, or garbage that happens to equal gen, which
// merely runs the general path for nothing) redo the file by the general path, overwriting
// everything; so the count pass's read of the file is skipped only for files where the result is
// already right.
template <int KIND>
__global__ __launch_bounds__(WG) void whitelist_spec16_kernel(const uint8_t* __restrict__ buf, int64_t n, int64_t cap,
                                                              int words, uint64_t* __restrict__ codes,
                                                              int64_t* __restrict__ starts, int32_t* __restrict__ lens,
                                                              uint8_t* __restrict__ gc, uint8_t* __restrict__ flags,
                                                              unsigned long long* __restrict__ d_nlines,
                                                              int32_t* __restrict__ d_maxlen,
                                                              unsigned* __restrict__ fail, unsigned gen) {
  constexpr int S = 17, L = 16;
  __shared__ uint8_t lut[256];
  __shared__ int s_stride;
  const int t = threadIdx.x;
  for (int c = t; c < 256; c += WG) lut[c] = lut_entry(KIND, c);
  if (file_stride(buf, n, &s_stride) != S) {  // (its barrier also covers the LUT)
    if (blockIdx.x == 0 && t == 0) atomicExch(fail, gen);
    return;
  }
  const int64_t nl = n / S, gend = nl < cap ? nl : (cap > 0 ? cap : 0);
  if (blockIdx.x == 0 && t == 0) {
    *d_nlines = (unsigned long long)nl;
    *d_maxlen = L;
  }
  bool ok = true;
  constexpr int U = 4;  // lines per thread per step, all their loads issued before any is used
  for (int64_t g0 = (int64_t)blockIdx.x * WG + t; g0 < nl; g0 += (int64_t)U * gridDim.x * WG) {
    uint32_t d[U][5];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t g = g0 + (int64_t)u * gridDim.x * WG, start = g * S;
      const uint32_t o = (uint32_t)(start & 3);
      if (g < nl && start - o + 20 <= n) {
        const uint32_t* w = reinterpret_cast<const uint32_t*>(buf + (start - o));
#pragma unroll
        for (int k = 0; k < 5; ++k) d[u][k] = w[k];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t g = g0 + (int64_t)u * gridDim.x * WG, start = g * S;
      if (g >= nl) break;
      const uint32_t o = (uint32_t)(start & 3);
      uint64_t code = 0;
      uint32_t gg = 0, fl = 0;
      bool done = false;
      if (start - o + 20 <= n) {
        uint32_t bad = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t x = __builtin_amdgcn_alignbyte(d[u][k + 1], d[u][k], o);
          const uint32_t uu = ((x >> 1) ^ (x >> 2)) & 0x03030303u;
          const uint32_t v = uu ^ ((uu >> 1) & 0x01010101u);
          bad |= __builtin_amdgcn_perm(0u, 0x47544341u, v) ^ x;
          const uint32_t y =
              __builtin_amdgcn_perm(0u, KIND == 2 ? v : __builtin_amdgcn_perm(0u, 0x03040102u, v), 0x00010203u);
          if (KIND == 2) {
            const uint32_t a = (y | (y >> 6)) & 0x000F000Fu;
            code = (code << 8) | ((a | (a >> 12)) & 0xFFu);
          } else {
            const uint32_t a = (y | (y >> 5)) & 0x003F003Fu;
            code = (code << 12) | ((a | (a >> 10)) & 0xFFFu);
          }
        }
        ok = ok && ((d[u][4] >> (8 * o)) & 0xFFu) == 0x0Au;  // byte 16 of the line: its '\n'
        if (!bad) {
          gg = (uint32_t)__popcll(code & (KIND == 2 ? 0x5555555555555555ull : 0x9249249249249249ull));
          done = true;
        }
      } else {
        ok = ok && buf[start + L] == 0x0Au;
      }
      if (!done) {  // another byte in the line (the LUT), or the file's last line: any '\n' breaks the stride
        for (int p = 0; p < L; ++p) ok = ok && buf[start + p] != 0x0Au;
        encode_line<KIND>(lut, buf + start, L, 1, &code, gg, fl);
      }
      if (g < gend) {
        codes[g * words] = code;  // (a 16-base code is one limb; wider rows get zero upper limbs)
        for (int w = 1; w < words; ++w) codes[g * words + w] = 0;
        starts[g] = start;
        lens[g] = L;
        if (gc) gc[g] = (uint8_t)gg;
        if (flags) flags[g] = (uint8_t)fl;
      }
    }
  }
  if (!ok) atomicExch(fail, gen);
}

extern "C" int sct_whitelist_encode(const uint8_t* d_buf, int64_t nbytes, int kind, int words, int64_t max_lines,
                                    uint64_t* d_codes, int64_t* d_starts, int32_t* d_lens, uint8_t* d_gc,
                                    uint8_t* d_flags, int64_t* d_nlines, int32_t* d_maxlen, void* stream) {
  SCT_CHECK(kind == 2 || kind == 3, "kind must be 2 or 3");
  SCT_CHECK(words >= 1 && d_nlines != nullptr && d_maxlen != nullptr, "bad arguments");
  SCT_CHECK(nbytes >= 0 && (nbytes == 0 || d_buf != nullptr), "bad buffer");
  SCT_CHECK(max_lines <= 0 || (d_codes && d_starts && d_lens), "NULL output");
  hipStream_t s = sct::as_stream(stream);
  if (nbytes == 0) {
    SCT_HIP(hipMemsetAsync(d_maxlen, 0, 4, s));
    SCT_HIP(hipMemsetAsync(d_nlines, 0, 8, s));
    return SCT_OK;
  }
  const int64_t ntiles = sct::ceil_div(nbytes, WTILE);
  // tile numbers stay below 2^32 / WG (the guard of ADVICE r4, kept for the encode pass's grid)
  SCT_CHECK(ntiles * WG < (1LL << 32), "buffer too large: %lld bytes (one launch covers < %lld)", (long long)nbytes,
            (long long)(((1LL << 32) / WG) * WTILE));
  const size_t tsb = (sct::tile_sums_bytes(ntiles, true) + 255) & ~(size_t)255;
  StreamBuf scratch;
  SCT_HIP(scratch.alloc(tsb + 256, s));
  const sct::TileSums ts = sct::tile_sums_at(scratch.p, ntiles, true, true);
  const int64_t cap = max_lines > 0 ? max_lines : 0;
  // 16-base lines are tried in one read first (whitelist_spec16_kernel): when the file is that
  // layout, the passes below return at once; else they redo it (SCT_TUNE_INGEST_SPEC = 0: never)
  unsigned* spec_fail = nullptr;
  static std::atomic<unsigned> g_spec_gen{0};
  unsigned gen = 0;
  if (nbytes % 17 == 0 && sct::tune(SCT_TUNE_INGEST_SPEC, 1) != 0) {
    spec_fail = reinterpret_cast<unsigned*>(reinterpret_cast<uint8_t*>(scratch.p) + tsb);
    gen = ++g_spec_gen;  // (a new value per call: the scratch word is not cleared)
    auto spec = kind == 2 ? whitelist_spec16_kernel<2> : whitelist_spec16_kernel<3>;
    const int64_t nl = nbytes / 17;
    const unsigned sg = (unsigned)std::max<int64_t>(1, std::min<int64_t>(sct::ceil_div(nl, 4 * WG), 8192));
    hipLaunchKernelGGL(spec, dim3(sg), dim3(WG), 0, s, d_buf, nbytes, cap, words, d_codes, d_starts, d_lens, d_gc, d_flags,
                       reinterpret_cast<unsigned long long*>(d_nlines), d_maxlen, spec_fail, gen);
    SCT_LAUNCH_CHECK();
  }
  // (no work depends on another workgroup here: a grid of resident slots without stopping the
  // scalar server, the occupancy looked up once)
  static const int64_t count_slots = [] {
    int dev = 0, cus = 256, per_cu = 0;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, wl_count_kernel, WG, 0) != hipSuccess || per_cu <= 0)
      per_cu = 4;
    return (int64_t)cus * per_cu;
  }();
  const unsigned cg = (unsigned)std::max<int64_t>(1, std::min<int64_t>(ntiles, count_slots));
  hipLaunchKernelGGL(wl_count_kernel, dim3(cg), dim3(WG), 0, s, d_buf, nbytes, ntiles, ts, d_maxlen,
                     (const unsigned*)spec_fail, gen);
  SCT_LAUNCH_CHECK();
  // up to 4,096 tiles (64 MiB) every encode workgroup reads the per-tile words itself (<= 16 per
  // thread) instead of waiting for a reduction launch
  const int direct = ntiles <= sct::tune(SCT_TUNE_INGEST_DIRECT, 4096) ? 1 : 0;
  if (!direct) {
    hipLaunchKernelGGL(sct::tile_sums_reduce_kernel, dim3((unsigned)sct::ceil_div(ntiles, 1024)), dim3(64), 0, s, ts,
                       ntiles, (const unsigned*)spec_fail, gen);
    SCT_LAUNCH_CHECK();
  }
  auto kern = kind == 2 ? whitelist_fused_kernel<2> : whitelist_fused_kernel<3>;
  // one range per resident slot (0.081 ms for config 5's whitelist; one 16 KiB tile per
  // workgroup 0.088, tools/ingest_tiles_ab.py); SCT_TUNE_INGEST_TILES > 0 fixes the range
  const int64_t knob = sct::tune(SCT_TUNE_INGEST_TILES, 0);
  const int64_t per_wg = knob > 0 ? knob : sct::ceil_div(ntiles, resident_slots((const void*)kern, ntiles));
  hipLaunchKernelGGL(kern, dim3((unsigned)sct::ceil_div(ntiles, per_wg)), dim3(WG), 0, s, d_buf, nbytes, ntiles,
                     per_wg, ts, direct, cap, words, d_codes, d_starts, d_lens, d_gc, d_flags,
                     reinterpret_cast<unsigned long long*>(d_nlines), d_maxlen, (const unsigned*)spec_fail, gen);
  SCT_LAUNCH_CHECK();
  return SCT_OK;
}

// Host convenience for Barcodes.from_whitelist: the file's bytes in, every line's [:-1]
// encoded (kind 2 TwoBit / 3 ThreeBit) as `words` limbs, plus each line's start, chopped
// length and flags (sct_encode's: bit 0 ambiguous base, bit 1 invalid byte).  Call with
// max_lines = 0 to learn nlines and the longest line (outputs untouched); then with
// room for nlines rows and words >= ceil(kind * longest / 64).
extern "C" int sct_whitelist_encode_host(const uint8_t* buf, int64_t nbytes, int kind, int words, int64_t max_lines,
                                         int64_t* nlines, int32_t* max_len, uint64_t* codes, int64_t* starts,
                                         int32_t* lens, uint8_t* flags) {
  SCT_CHECK(kind == 2 || kind == 3, "kind must be 2 or 3");
  SCT_CHECK(nlines && max_len && words >= 1, "bad arguments");
  SCT_CHECK(nbytes >= 0 && (nbytes == 0 || buf), "bad buffer");
  sct::HostStage* st = sct::host_stage();
  if (!st) return SCT_E_HIP;
  // device: the file, then (a filling call) starts, lens, codes, flags, then the count and the longest
  const int64_t cap = max_lines > 0 ? max_lines : 0;
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t oS = al((size_t)nbytes), oL = oS + al((size_t)cap * 8), oC = oL + al((size_t)cap * 4);
  const size_t oF = oC + al((size_t)cap * words * 8), oN = oF + al((size_t)cap), total = oN + 256;
  if (int rc = sct::stage_reserve(st, 64, total); rc != SCT_OK) return rc;
  uint8_t* d = st->dev;
  if (nbytes) SCT_HIP(hipMemcpyAsync(d, buf, (size_t)nbytes, hipMemcpyHostToDevice, st->stream));
  int64_t* d_n = reinterpret_cast<int64_t*>(d + oN);
  int32_t* d_mx = reinterpret_cast<int32_t*>(d + oN + 8);
  int rc = sct_whitelist_encode(d, nbytes, kind, words, cap, reinterpret_cast<uint64_t*>(d + oC),
                                reinterpret_cast<int64_t*>(d + oS), reinterpret_cast<int32_t*>(d + oL), nullptr,
                                d + oF, d_n, d_mx, st->stream);
  if (rc != SCT_OK) return rc;
  int64_t* h = reinterpret_cast<int64_t*>(st->pinned);
  SCT_HIP(hipMemcpyAsync(h, d_n, 16, hipMemcpyDeviceToHost, st->stream));
  SCT_HIP(hipStreamSynchronize(st->stream));
  const int64_t n = h[0];
  *nlines = n;
  *max_len = n ? reinterpret_cast<int32_t*>(h + 1)[0] : 0;
  if (cap < n || n == 0) return SCT_OK;  // a sizing call (or an empty file): outputs untouched
  SCT_CHECK(codes && starts && lens && flags, "NULL output");
  SCT_CHECK((int64_t)kind * *max_len <= (int64_t)words * 64, "words %d too few for lines of %d bases", words,
            *max_len);
  SCT_HIP(hipMemcpyAsync(codes, d + oC, (size_t)n * words * 8, hipMemcpyDeviceToHost, st->stream));
  SCT_HIP(hipMemcpyAsync(starts, d + oS, (size_t)n * 8, hipMemcpyDeviceToHost, st->stream));
  SCT_HIP(hipMemcpyAsync(lens, d + oL, (size_t)n * 4, hipMemcpyDeviceToHost, st->stream));
  SCT_HIP(hipMemcpyAsync(flags, d + oF, (size_t)n, hipMemcpyDeviceToHost, st->stream));
  SCT_HIP(hipStreamSynchronize(st->stream));
  return SCT_OK;
}
