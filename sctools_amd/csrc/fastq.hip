// FASTQ embedded-barcode extraction on gfx950.
//
// Replaces the per-record Python path that feeds barcodes into the hot path:
//   reader.Reader.__iter__            (src/sctools/reader.py:56-85)   lines of each file, in order
//   fastq.Reader.record_grouper       (src/sctools/fastq.py:143-150)  4 consecutive lines = 1 record
//   fastq.Record.name setter          (src/sctools/fastq.py:31-38)    name must start with '@'
//   EmbeddedBarcodeGenerator.__iter__ / extract_barcode (src/sctools/fastq.py:181-200):
//       record.sequence[start:end], record.quality[start:end]
// with the TenXV2 spans of platform.py:36-38 as the typical use.
//
// Semantics kept exactly: a line includes its newline, so a slice past the end of a short
// read includes the '\n'; a file's last line may lack one; files are concatenated line
// streams (a record may span two files) and an incomplete trailing record is dropped.
// Mode 'rb' splits lines at '\n' only; mode 'r' (text) at '\n', "\r\n" and a lone '\r',
// each read back as '\n' (Python's universal newlines), and only ASCII input is accepted.
//
// Device layout: the files' bytes concatenated in one buffer, read in 8 KiB tiles (32 bytes
// per thread as two 16-byte loads, SWAR byte compares).  Two passes: count_kernel counts each tile's line
// terminators and an exclusive scan gives every tile its first line number (the index);
// extract2_kernel finds the terminators again, numbers them, and for each one that starts a
// record's name / sequence / quality line checks the '@' or copies that line's slices.
// No per-line array is ever stored.
#include <hipcub/hipcub.hpp>

#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <utility>
#include <mutex>
#include <vector>

#include "sct_common.h"
#include "encode_common.h"
#include "tile_prefix.h"

namespace {

constexpr int WG = 256;
constexpr int TILE = 8192;  // bytes per thread-block tile
constexpr int TB = TILE / WG;  // bytes per thread
constexpr int SEG = TB / 16;   // 16-B loads per thread

#ifndef SCT_FQ_ABL
#define SCT_FQ_ABL 0  // timing-only ablations of the extraction kernels (tools/build_fq_abl.sh; 5 = the
                      // per-line row / length / code stores into an LDS sink instead of memory)
#endif

struct Files {
  const int64_t* ends;  // cumulative end offsets, nfiles entries
  int nfiles;
};

// file f ends at e (> its start) without a terminator on its last byte -> virtual terminator
__device__ __forceinline__ bool virtual_end(const uint8_t* __restrict__ buf, int64_t n, Files fs, int f,
                                            int text) {
  const int64_t e = fs.ends[f], s = f ? fs.ends[f - 1] : 0;
  if (e <= s) return false;
  // a "\r\n" split across the file boundary is two files' bytes: only bytes of this file count
  const uint8_t c = buf[e - 1];
  return !(c == '\n' || (text && c == '\r'));
}

// Each 16-byte load: terminators as a 16-bit mask; a thread owns SEG of them (thread_span);
// a tile = 256 threads = 8 KiB (half the barriers and scans per byte of 4 KiB tiles: 0.87 vs
// 1.31 ms per 20M-record extraction).
// Terminators of the thread's bytes as a 16-bit mask (bit j = byte p0 + j), found with
// SWAR byte compares on the four 32-bit words; text mode also needs the byte before and
// after the span (a '\r' before '\n' is part of "\r\n", a lone '\r' is a terminator).
__device__ __forceinline__ uint32_t eq_bytes(uint32_t w, uint32_t pat) {
  // bit 7 of each byte set iff that byte equals the pattern byte (exact, no carries)
  const uint32_t x = w ^ pat;
  return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
}
__device__ __forceinline__ uint32_t byte_mask4(uint32_t hi_bits) {  // bit 7 of byte k -> bit k
  // one multiply: (hi >> 7) * (2^28 + 2^21 + 2^14 + 2^7) puts byte k's bit at 28 + k and every
  // other partial product at a distinct bit below 24 or past 31 (tests/test_swar_host.py)
  return ((hi_bits >> 7) * 0x10204080u) >> 28;
}

// the 16 bytes at p0 (zero past n)
__device__ __forceinline__ uint4 load16(const uint8_t* __restrict__ buf, int64_t n, int64_t p0) {
  if (p0 + 16 <= n) return *reinterpret_cast<const uint4*>(buf + p0);
  uint32_t w[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint32_t x = 0;
    for (int b = 0; b < 4; ++b)
      if (p0 + 4 * k + b < n) x |= (uint32_t)buf[p0 + 4 * k + b] << (8 * b);
    w[k] = x;
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// terminator mask of the 16 bytes v loaded from p0
__device__ __forceinline__ uint32_t load_mask(const uint8_t* __restrict__ buf, int64_t n, int64_t p0,
                                              int text, uint32_t* kinds_crlf, uint32_t* nonascii, uint4 v) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  const uint32_t valid = p0 + 16 <= n ? 0xFFFFu : (uint32_t)((1u << (n - p0)) - 1u);
  uint32_t lf = 0, cr = 0, na = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    lf |= byte_mask4(eq_bytes(w[k], 0x0A0A0A0Au)) << (4 * k);
    if (text) cr |= byte_mask4(eq_bytes(w[k], 0x0D0D0D0Du)) << (4 * k);
    na |= w[k] & 0x80808080u;
  }
  lf &= valid;
  cr &= valid;
  uint32_t m = lf, crlf = 0;
  if (text) {
    const uint32_t cr_prev = (p0 > 0 && buf[p0 - 1] == '\r') ? 1u : 0u;  // byte before the span
    const uint32_t lf_next = (p0 + 16 < n && buf[p0 + 16] == '\n') ? 1u : 0u;
    crlf = lf & ((cr << 1) | cr_prev);                    // '\n' preceded by '\r'
    const uint32_t lone_cr = cr & ~((lf >> 1) | (lf_next << 15));  // '\r' not followed by '\n'
    m = lf | lone_cr;
  }
  *kinds_crlf = crlf;
  *nonascii = na;
  return m;
}

// file f's end e lies in (p0, p0 + 16] and its last byte is not a terminator -> virtual
// terminator at e; returns the in-span offset e - p0 - 1 of its last byte, or -1
__device__ __forceinline__ int virtual_in(const uint8_t* __restrict__ buf, int64_t n, Files fs,
                                          int64_t p0, int text) {
  int lo = 0, hi = fs.nfiles;  // first file with end > p0
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (fs.ends[mid] <= p0) lo = mid + 1; else hi = mid;
  }
  for (int f = lo; f < fs.nfiles && fs.ends[f] <= p0 + 16; ++f)
    if (virtual_end(buf, n, fs, f, text)) return (int)(fs.ends[f] - p0 - 1);
  return -1;
}

// A thread's TB bytes at p0 (SEG 16-B segments v): terminator mask m, "\r\n" mask crlf and
// virtual file-end mask vbits (bit j = byte p0 + j; a virtual end is put on the file's last
// byte, never a terminator itself), and the non-ASCII bits of the bytes.
struct Span {
  uint32_t m, crlf, vbits, na;
};
__device__ __forceinline__ Span thread_span(const uint8_t* __restrict__ buf, int64_t n, Files fs, int text,
                                            int64_t p0, const uint4* v, bool ends_here) {
  Span s{0, 0, 0, 0};
#pragma unroll
  for (int k = 0; k < SEG; ++k) {
    const int64_t q = p0 + 16 * k;
    if (q >= n) break;
    uint32_t cr, na;
    s.m |= load_mask(buf, n, q, text, &cr, &na, v[k]) << (16 * k);
    s.crlf |= cr << (16 * k);
    s.na |= na;
    if (ends_here) {
      const int x = virtual_in(buf, n, fs, q, text);
      if (x >= 0) s.vbits |= 1u << (16 * k + x);
    }
  }
  return s;
}

// A workgroup's walk over increasing tile starts t0: f = the first file ending after t0 (loads
// of uniform addresses: scalar), so a tile holding no file end (almost all of them) skips the
// per-thread virtual-terminator search.
struct FileCursor {
  int f = 0;
  __device__ __forceinline__ bool advance(Files fs, int64_t t0) {
    while (f < fs.nfiles && fs.ends[f] <= t0) ++f;
    return f < fs.nfiles && fs.ends[f] <= t0 + TILE + 16;
  }
};

// Per tile: its terminator count, and its first terminator (in-tile offset << 2 | 1 if
// virtual | 2 if "\r\n"; ~0 if none) -- the end of the previous tile's last line.
// Persistent: a workgroup walks tiles blockIdx.x, + gridDim.x, ... with the next tile's
// 16 bytes per thread loaded before this tile is reduced (one load in flight per thread
// while it works: a tile per workgroup left the loads latency-bound).
__global__ __launch_bounds__(WG) void count_kernel(const uint8_t* __restrict__ buf, int64_t n, Files fs,
                                                   int text, unsigned long long* __restrict__ counts,
                                                   uint32_t* __restrict__ first,
                                                   unsigned* __restrict__ flags, int64_t ntiles) {
  using BR = hipcub::BlockReduce<uint32_t, WG>;
  __shared__ typename BR::TempStorage tmp;
  int64_t tile = blockIdx.x;
  uint4 cur[SEG], nxt[SEG];
#pragma unroll
  for (int k = 0; k < SEG; ++k)
    cur[k] = tile < ntiles ? load16(buf, n, tile * TILE + (int64_t)threadIdx.x * TB + 16 * k) : make_uint4(0, 0, 0, 0);
  FileCursor fc;
  for (; tile < ntiles; tile += gridDim.x) {
    const int64_t nt = tile + gridDim.x;
#pragma unroll
    for (int k = 0; k < SEG; ++k)
      nxt[k] = nt < ntiles ? load16(buf, n, nt * TILE + (int64_t)threadIdx.x * TB + 16 * k) : make_uint4(0, 0, 0, 0);
    const int64_t p0 = tile * TILE + (int64_t)threadIdx.x * TB;
    const bool ends_here = fc.advance(fs, tile * TILE);  // wave-uniform: a file end in this tile
    uint32_t c = 0, na = 0, f = ~0u;
    if (p0 < n) {
      const Span sp = thread_span(buf, n, fs, text, p0, cur, ends_here);
      na = sp.na;
      const uint32_t bits = sp.m | sp.vbits;
      c = __popc(bits);
      if (bits) {
        const int j = __ffs(bits) - 1;
        f = (sp.m >> j & 1u) ? ((uint32_t)(threadIdx.x * TB + j) << 2) | ((sp.crlf >> j & 1u) ? 2u : 0u)
                             : ((uint32_t)(threadIdx.x * TB + j + 1) << 2) | 1u;
      }
    }
    __syncthreads();  // the previous tile's reductions are done with tmp
    const uint32_t tot = BR(tmp).Sum(c);
    __syncthreads();
    const uint32_t fmin = BR(tmp).Reduce(f, hipcub::Min());
    if (na) atomicOr(flags, 1u);
    if (threadIdx.x == 0) {
      counts[tile] = tot;
      first[tile] = fmin;
    }
#pragma unroll
    for (int k = 0; k < SEG; ++k) cur[k] = nxt[k];
  }
}

// A line as the reference sees it: content [start, content_end), then '\n' when nl.  From a
// line start, scan at most `need` bytes for its terminator ('\n'; in text mode also '\r',
// whether of "\r\n" or lone) without crossing the end of the file that holds `start`.
struct Line {
  int64_t start, content_end;
  int nl;
};

__device__ __forceinline__ Line scan_line(const uint8_t* __restrict__ buf, int64_t n, Files fs,
                                          int64_t start, int need, int text) {
  int lo = 0, hi = fs.nfiles;  // the file holding `start`: first end > start
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (fs.ends[mid] <= start) lo = mid + 1; else hi = mid;
  }
  const int64_t fe = lo < fs.nfiles ? fs.ends[lo] : n;
  const int64_t lim = start + need < fe ? start + need : fe;
  Line L{start, lim, 1};
  for (int64_t i = start; i < lim; ++i) {
    const uint8_t c = buf[i];
    if (c == '\n' || (text && c == '\r')) {
      L.content_end = i;
      return L;
    }
  }
  // no terminator in the window: the line is longer than needed (content_end = lim is
  // enough), or it is the file's unterminated last line
  if (lim == fe) L.nl = 0;
  return L;
}

// One pass over the buffer, a tile per workgroup:
//  1. each thread finds its 16 bytes' terminators (as count_kernel) and the block scan
//     numbers them; their in-tile offsets go to LDS in byte order (bit 13 = virtual file
//     end: the next line starts at the end and the line has no '\n'; bit 14 = "\r\n");
//  2. the line after terminator t (global number g+1) belongs to record (g+1)/4: a name
//     line (0) must start with '@' (fastq.py:35-36); for a sequence (1) or quality (3)
//     line, one item per line finds the line's end at the tile's next terminator
//     (for the tile's last line: the next tile's first, or a short scan) and copies its
//     slice (rows inside the tile from the tile's LDS copy).
// Record 0's name line starts at byte 0, checked by thread 0 of tile 0.
constexpr int MAX_SPANS = 8;
struct Spans {
  int n, max_end, width;  // width = sum of the spans' widths
  int start[MAX_SPANS], end[MAX_SPANS];
  int64_t prefix[MAX_SPANS];  // sum of the widths of the spans before k
};

constexpr int MAX_TERM = TILE + 16;  // terminators a tile can hold (+ virtual file ends)

// The extraction (round 2: fewer LDS bytes and one barrier fewer per tile than the first
// version, which kept 32-bit terminators and an action array): terminators as
// 16-bit tile offsets (bit 13 = virtual file end, bit 14 = "\r\n"; 8 KB), no action array --
// a copy item (line a) finds its line from the terminators around it (the line after the
// tile's (te0 + 2a)-th terminator; te0 = 1 when the tile's first terminator number is odd) and
// copies every span of it in turn -- so the name checks and the copies run in one phase after
// the terminators are written.  13 KB of LDS: 7 resident workgroups per CU (4 for the first
// version).  Round 3: one item per line instead of per (line, span), so a line's end is found
// once for all its spans: 20M records 1.33-1.35 -> 1.16-1.21 ms.
constexpr uint16_t T16_OFF = 0x3FFF, T16_VIRT = 1u << 14, T16_CRLF = 1u << 15;
static_assert(TILE + 16 <= T16_OFF, "16-bit terminator offsets");

__global__ __launch_bounds__(WG) void extract2_kernel(const uint8_t* __restrict__ buf, int64_t n, Files fs,
                                                      int text, const unsigned long long* __restrict__ offsets,
                                                      const uint32_t* __restrict__ first, int64_t ntiles,
                                                      int64_t nrec, Spans sp, uint8_t* __restrict__ seq_out,
                                                      uint8_t* __restrict__ qual_out,
                                                      int32_t* __restrict__ seq_len,
                                                      int32_t* __restrict__ qual_len,
                                                      unsigned long long* __restrict__ first_bad) {
  __shared__ uint16_t term[MAX_TERM];
  __shared__ uint4 tile_bytes[TILE / 16];  // the tile itself: slices inside it copy from LDS
  using BS = hipcub::BlockScan<uint32_t, WG>;
  __shared__ typename BS::TempStorage tmp;
  int64_t tile = blockIdx.x;
  uint4 cur[SEG], nxt[SEG];
#pragma unroll
  for (int k = 0; k < SEG; ++k)
    cur[k] = tile < ntiles ? load16(buf, n, tile * TILE + (int64_t)threadIdx.x * TB + 16 * k) : make_uint4(0, 0, 0, 0);
  unsigned long long g0_cur = tile < ntiles ? offsets[tile] : 0ull;
  uint32_t nf_cur = tile + 1 < ntiles ? first[tile + 1] : ~0u;
  FileCursor fc;
  const uint8_t* tile8 = reinterpret_cast<const uint8_t*>(tile_bytes);
  const uint32_t* tile32 = reinterpret_cast<const uint32_t*>(tile_bytes);
  for (; tile < ntiles; tile += gridDim.x) {
    const int64_t ntl = tile + gridDim.x;
#pragma unroll
    for (int k = 0; k < SEG; ++k)
      nxt[k] = ntl < ntiles ? load16(buf, n, ntl * TILE + (int64_t)threadIdx.x * TB + 16 * k) : make_uint4(0, 0, 0, 0);
    const unsigned long long g0_nxt = ntl < ntiles ? offsets[ntl] : 0ull;
    const uint32_t nf_nxt = ntl + 1 < ntiles ? first[ntl + 1] : ~0u;
    const int64_t t0 = tile * TILE;
    const int64_t p0 = t0 + (int64_t)threadIdx.x * TB;
    const bool ends_here = fc.advance(fs, t0);
    Span spn{0, 0, 0, 0};
    if (p0 < n) spn = thread_span(buf, n, fs, text, p0, cur, ends_here);
    __syncthreads();  // the previous tile's readers of tile_bytes / term / tmp are done
#pragma unroll
    for (int k = 0; k < SEG; ++k) {
      tile_bytes[threadIdx.x * SEG + k] = p0 + 16 * k < n ? cur[k] : make_uint4(0, 0, 0, 0);
      cur[k] = nxt[k];
    }
    const uint32_t tbits = spn.m | spn.vbits;
    uint32_t pre, ntile;
    BS(tmp).ExclusiveSum((uint32_t)__popc(tbits), pre, ntile);
    {
      uint32_t bits = tbits;
      uint32_t at = pre;
      while (bits) {
        const int j = __ffs(bits) - 1;
        bits &= bits - 1;
        const uint32_t off = (uint32_t)(threadIdx.x * TB + j);
        term[at++] = (spn.m >> j & 1u) ? (uint16_t)(off | ((spn.crlf >> j & 1u) ? T16_CRLF : 0u))
                                       : (uint16_t)((off + 1) | T16_VIRT);  // the file ends after byte off
      }
    }
    __syncthreads();
    const int64_t g0 = (int64_t)g0_cur;  // global number of the tile's first terminator
    const uint32_t nf = nf_cur;
    if (tile == 0 && threadIdx.x == 0 && nrec > 0 && buf[0] != '@') atomicMin(first_bad, 0ull);
    // terminators of the tile that belong to records < nrec: [0, tmax)
    const int64_t lim_g = 4 * nrec - 1;  // terminators beyond the last record's line 3 end nothing
    const int tmax = (int)(g0 + ntile <= lim_g ? ntile : (lim_g > g0 ? lim_g - g0 : 0));
    // name lines: after terminators g = 3 (mod 4)
    for (int t = (int)((3 - (g0 & 3)) & 3) + 4 * (int)threadIdx.x; t < tmax; t += 4 * WG) {
      const uint32_t e = term[t];
      const int64_t o = (int64_t)(e & T16_OFF) + ((e & T16_VIRT) ? 0 : 1);  // the line's start in the tile
      const uint8_t ch = o < TILE ? tile8[o] : buf[t0 + o];
      if (ch != '@') atomicMin(first_bad, (unsigned long long)((g0 + t + 1) >> 2));
    }
    // sequence / quality lines: after even terminators; one item per line, its spans in turn
    // (the line's end is found once for all of them)
    const int te0 = (int)(g0 & 1);
    const int nact = tmax > te0 ? (tmax - te0 + 1) / 2 : 0;
    for (int a = threadIdx.x; a < nact; a += WG) {
      const int t = te0 + 2 * a;
      const int64_t line = g0 + t + 1, rec = line >> 2;
      const bool is_seq = (line & 3) == 1;
      const uint32_t e = term[t];
      const int start = (int)(e & T16_OFF) + ((e & T16_VIRT) ? 0 : 1);  // <= TILE
      int64_t cend;  // content end relative to the tile start
      int nl;
      if (t + 1 < (int)ntile) {  // the line ends at the tile's next terminator
        const uint32_t f = term[t + 1];
        cend = (int64_t)(f & T16_OFF) - ((f & T16_CRLF) ? 1 : 0);
        nl = (f & T16_VIRT) ? 0 : 1;
      } else if (nf != ~0u) {  // the tile's last line ends at the next tile's first terminator
        cend = TILE + (int64_t)(nf >> 2) - ((nf & 2u) ? 1 : 0);
        nl = (nf & 1u) ? 0 : 1;
      } else {  // no terminator in the next tile either: scan (max_end bytes, within its file)
        const int64_t next = t0 + start;
        int lo = 0, hi = fs.nfiles;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (fs.ends[mid] <= next) lo = mid + 1; else hi = mid;
        }
        const int64_t fe = lo < fs.nfiles ? fs.ends[lo] : n;
        const int64_t lim = next + sp.max_end < fe ? next + sp.max_end : fe;
        cend = lim - t0;
        nl = lim == fe ? 0 : 1;  // longer than the window: its end is irrelevant
        for (int64_t i = next; i < lim; ++i) {
          const uint8_t ch = buf[i];
          if (ch == '\n' || (text && ch == '\r')) {
            cend = i - t0;
            nl = 1;
            break;
          }
        }
      }
      int32_t* len = is_seq ? seq_len : qual_len;
      uint8_t* out = is_seq ? seq_out : qual_out;
      const int64_t clen = cend - start, llen = clen + nl;
      for (int k = 0; k < sp.n; ++k) {
        const int64_t sa = sp.start[k] < llen ? sp.start[k] : llen, sb = sp.end[k] < llen ? sp.end[k] : llen;
        if (len) len[k * nrec + rec] = (int32_t)(sb - sa);
        if (!out) continue;
        const int w = sp.end[k] - sp.start[k];
        uint8_t* o = out + sp.prefix[k] * nrec + rec * w;
        const uint8_t* src = buf + t0 + start;
        // fast path: a whole-width slice inside the line's content, a row of whole dwords:
        // aligned dword loads + byte-align funnel shifts, dword stores
        const int64_t s0 = t0 + start + sa;
        const int64_t base = s0 & ~3LL;
        const int nd = w / 4;
        if (sb - sa == w && sb <= clen && (w & 3) == 0 && w <= 64 && base + 4 * (nd + 1) <= n &&
            ((uintptr_t)o & 3) == 0) {
          // rows inside the tile read its LDS copy; the rest (lines running past it) read L2
          const uint32_t* d = base + 4 * (nd + 1) <= t0 + TILE ? tile32 + ((base - t0) >> 2)
                                                               : reinterpret_cast<const uint32_t*>(buf + base);
          const uint32_t sh = (uint32_t)(s0 & 3);
          uint32_t* od = reinterpret_cast<uint32_t*>(o);
          if (nd == 4 && ((uintptr_t)o & 15) == 0) {
            const uint32_t x0 = d[0], x1 = d[1], x2 = d[2], x3 = d[3], x4 = d[4];
            *reinterpret_cast<uint4*>(o) =
                make_uint4(__builtin_amdgcn_alignbyte(x1, x0, sh), __builtin_amdgcn_alignbyte(x2, x1, sh),
                           __builtin_amdgcn_alignbyte(x3, x2, sh), __builtin_amdgcn_alignbyte(x4, x3, sh));
            continue;
          }
          if (nd == 2 && ((uintptr_t)o & 7) == 0) {
            const uint32_t x0 = d[0], x1 = d[1], x2 = d[2];
            *reinterpret_cast<uint2*>(o) =
                make_uint2(__builtin_amdgcn_alignbyte(x1, x0, sh), __builtin_amdgcn_alignbyte(x2, x1, sh));
            continue;
          }
          uint32_t lo = d[0];
          for (int q2 = 0; q2 < nd; ++q2) {
            const uint32_t hi = d[q2 + 1];
            od[q2] = __builtin_amdgcn_alignbyte(hi, lo, sh);
            lo = hi;
          }
          continue;
        }
#pragma unroll 8
        for (int j = 0; j < w; ++j) {
          const int64_t i = sa + j;
          o[j] = i < sb ? (i < clen ? src[i] : (uint8_t)'\n') : (uint8_t)0;
        }
      }
    }
    g0_cur = g0_nxt;
    nf_cur = nf_nxt;
  }
}

// ---------------------------------------------------------------- without an index (round 4)
// sct_fastq_extract_fused: fq_count_kernel (one 8 KiB tile per workgroup: a one-pass grid streams
// the buffer at the copy rate, where the persistent count_kernel loop stayed near 4 TB/s) writes
// every tile's terminator count and first terminator (count_kernel's encoding) and the non-ASCII
// flag; tile_sums_reduce_kernel sums the counts into the coarse levels of tile_prefix.h; then
// fastq_range_kernel gives each workgroup a contiguous range of tiles: it takes its first tile's
// line number and the total line count from the tile sums once, and walks its range carrying the
// line number (extract2_kernel's per-tile work, next tile's bytes loaded while this one is worked).
// No scan launch, no host synchronisation, and no atomics on shared words: publishing into the
// coarse levels with atomics cost 608 us for 1.38 GB (every tile in flight adds to one word).
__global__ __launch_bounds__(WG) void fq_count_kernel(const uint8_t* __restrict__ buf, int64_t n, Files fs, int text,
                                                      sct::TileSums ts, uint32_t* __restrict__ first,
                                                      unsigned* __restrict__ flags) {
  const int64_t tile = blockIdx.x, t0 = tile * TILE, p0 = t0 + (int64_t)threadIdx.x * TB;
  uint4 cur[SEG];
#pragma unroll
  for (int k = 0; k < SEG; ++k) cur[k] = load16(buf, n, p0 + 16 * k);
  bool ends_here;
  {
    int lo = 0, hi = fs.nfiles;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (fs.ends[mid] <= t0) lo = mid + 1; else hi = mid;
    }
    ends_here = lo < fs.nfiles && fs.ends[lo] <= t0 + TILE + 16;
  }
  uint32_t c = 0, na = 0, f = ~0u;  // (a tile holds at most 8,192 terminators)
  if (!text && !ends_here && p0 + TB <= n) {
    // binary mode, no file end near the tile, a whole span: count the '\n' bytes straight from
    // the SWAR zero-byte bits (no per-byte mask: the count pass was VALU-bound, PMC 0.97 busy)
#pragma unroll
    for (int k = 0; k < SEG; ++k) {
      const uint32_t w[4] = {cur[k].x, cur[k].y, cur[k].z, cur[k].w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t hi = eq_bytes(w[q], 0x0A0A0A0Au) & 0x80808080u;
        c += __popc(hi);
        na |= w[q];
        if (hi && f == ~0u) f = (uint32_t)(threadIdx.x * TB + 16 * k + 4 * q + (__builtin_ctz(hi) >> 3)) << 2;
      }
    }
    na &= 0x80808080u;
  } else if (p0 < n) {
    const Span sp = thread_span(buf, n, fs, text, p0, cur, ends_here);
    const uint32_t bits = sp.m | sp.vbits;
    c = __popc(bits);
    na = sp.na;
    if (bits) {
      const int j = __ffs(bits) - 1;
      f = (sp.m >> j & 1u) ? ((uint32_t)(threadIdx.x * TB + j) << 2) | ((sp.crlf >> j & 1u) ? 2u : 0u)
                           : ((uint32_t)(threadIdx.x * TB + j + 1) << 2) | 1u;
    }
  }
  if (na) atomicOr(flags, 1u);
#pragma unroll
  for (int o = 32; o; o >>= 1) {
    c += __shfl_xor(c, o);
    f = min(f, (uint32_t)__shfl_xor(f, o));
  }
  __shared__ uint32_t wc[WG / 64];
  __shared__ uint32_t wf[WG / 64];
  if ((threadIdx.x & 63) == 0) {
    wc[threadIdx.x >> 6] = c;
    wf[threadIdx.x >> 6] = f;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < WG / 64; ++w) {
      c += wc[w];
      f = min(f, wf[w]);
    }
    sct::tile_publish(ts, tile, c, -1);
    first[tile] = f;
  }
}

// The per-tile work after the tile's terminators are in LDS (term, in byte order; the tile's
// bytes in tile8 / tile32, and `head` bytes of the next tile after them): the '@' check of every
// name line and every sequence / quality line's span slices (one item per line, its spans in
// turn; rows of records >= cap skipped).  Terminators [0, tmax) end lines of records that count
// (tmax < ntile drops an incomplete trailing record); g0 = the tile's first terminator's global
// number; nf = the next tile's first terminator (count_kernel's encoding), or ~0u: the tile's last
// line is then scanned for, in LDS when it ends within the staged head.
struct TileOut {
  uint8_t* seq_out;
  uint8_t* qual_out;
  int32_t* seq_len;
  int32_t* qual_len;
  uint64_t* codes0;
  uint8_t* gc0;
  uint8_t* flags0;
  int code_kind;
  uint64_t gc_mask;
  int64_t cap;
  unsigned long long* d_status;
};

// The 16 bytes at tile-relative offset s (>= 0): from the staged tile when lds (the 5-dword window
// lies in LDS), else from global memory (gt = the tile's first dword; the window lies in the buffer).
// One branch per window, not per dword: a per-dword LDS-or-global select compiled to a masked
// branch and a wait around every load.
__device__ __forceinline__ uint4 bytes16_at(lds_u32* tile32, const uint32_t* __restrict__ gt, int s, bool lds) {
  const int d = s >> 2;
  const uint32_t sh = (uint32_t)(s & 3);
  uint32_t x0, x1, x2, x3, x4;
  if (lds) {
    x0 = tile32[d], x1 = tile32[d + 1], x2 = tile32[d + 2], x3 = tile32[d + 3], x4 = tile32[d + 4];
  } else {
    x0 = gt[d], x1 = gt[d + 1], x2 = gt[d + 2], x3 = gt[d + 3], x4 = gt[d + 4];
  }
  return make_uint4(__builtin_amdgcn_alignbyte(x1, x0, sh), __builtin_amdgcn_alignbyte(x2, x1, sh),
                    __builtin_amdgcn_alignbyte(x3, x2, sh), __builtin_amdgcn_alignbyte(x4, x3, sh));
}

// the first m (1..16) bytes of y to o in pieces of G bytes (G: the largest of 16 / 8 / 4 / 2 / 1
// dividing the row width and the rows' base address; m is a multiple of G; both uniform)
#if SCT_FQ_ABL == 5  // the per-line stores into an LDS sink: the same work, no global stores
__device__ __forceinline__ void abl_sink(uint4 y) {
  __shared__ uint4 sink[64];
  sink[threadIdx.x & 63] = y;
}
#endif

__device__ __forceinline__ void store_row16(uint8_t* o, const uint4 y, int m, int G) {
#if SCT_FQ_ABL == 5
  abl_sink(make_uint4(y.x ^ (uint32_t)(uintptr_t)o, y.y ^ (uint32_t)m, y.z ^ (uint32_t)G, y.w));
  return;
#endif
  const uint32_t d[4] = {y.x, y.y, y.z, y.w};
  if (G == 16) {
    *reinterpret_cast<uint4*>(o) = y;
  } else if (G == 8) {
    *reinterpret_cast<uint2*>(o) = make_uint2(d[0], d[1]);
    if (m > 8) *reinterpret_cast<uint2*>(o + 8) = make_uint2(d[2], d[3]);
  } else if (G == 4) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (4 * j < m) reinterpret_cast<uint32_t*>(o)[j] = d[j];
  } else if (G == 2) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (2 * j < m) reinterpret_cast<uint16_t*>(o)[j] = (uint16_t)(d[j >> 1] >> (16 * (j & 1)));
  } else {
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (j < m) o[j] = (uint8_t)(d[j >> 2] >> (8 * (j & 3)));
  }
}

// r (1..4) bases of the dword w, MSB-first onto code: lines.hip encode_line1's SWAR (A/C/G/T upper
// case exactly), or -- when the dword holds any other byte -- its r bytes through the LUT (flags
// into fl), from the same register
__device__ __forceinline__ void enc_bases(uint32_t w, int r, int kind, const uint8_t* lut, uint64_t& code,
                                          uint32_t& fl) {
  const uint32_t x = ((w >> 1) ^ (w >> 2)) & 0x03030303u;
  const uint32_t v = x ^ ((x >> 1) & 0x01010101u);
  const uint32_t keep = r >= 4 ? ~0u : (1u << (8 * r)) - 1u;
  if ((__builtin_amdgcn_perm(0u, 0x47544341u, v) ^ w) & keep) {  // "ACTG"[v] != some byte
#pragma unroll
    for (int b = 0; b < 4; ++b)
      if (b < r) {
        const uint32_t e = lut[(w >> (8 * b)) & 0xFFu];
        code = (code << kind) | (e & 7u);
        fl |= e;
      }
  } else if (kind == 2) {
    const uint32_t y = __builtin_amdgcn_perm(0u, v, 0x00010203u);
    const uint32_t a = (y | (y >> 6)) & 0x000F000Fu, pk = (a | (a >> 12)) & 0xFFu;
    code = (code << (2 * r)) | (pk >> (2 * (4 - r)));
  } else {
    const uint32_t y = __builtin_amdgcn_perm(0u, __builtin_amdgcn_perm(0u, 0x03040102u, v), 0x00010203u);
    const uint32_t a = (y | (y >> 5)) & 0x003F003Fu, pk = (a | (a >> 10)) & 0xFFFu;
    code = (code << (3 * r)) | (pk >> (3 * (4 - r)));
  }
}

// One sequence / quality line's spans (NS > 0: that many, unrolled -- the span table in scalar
// registers; 0: sp.n in a loop).  The line starts at tile offset `start`, its content is clen bytes,
// llen with the '\n'.  A whole-width slice inside the content (the usual case) goes 16 bytes at a
// time from the staged tile (lines crossing the tile end: from global memory) to its row in pieces
// as wide as the row layout allows, span 0 of a sequence line TwoBit / ThreeBit-encoded from the
// same registers (SWAR; the LUT for the dwords holding other bytes); any other slice byte by byte
// ('\n' past the content, zero padding past the line, as the reference's slice of the line).
template <int NS>
__device__ __forceinline__ void line_spans(const Spans& sp, const TileOut& to, bool is_seq, int64_t rec, int start,
                                           int clen, int llen, lds_u32* tile32, const uint8_t* lut,
                                           const uint8_t* __restrict__ buf, int64_t n, int64_t t0, int lim_lds) {
  int32_t* len = is_seq ? to.seq_len : to.qual_len;
  uint8_t* out = is_seq ? to.seq_out : to.qual_out;
  const uint32_t* gt = reinterpret_cast<const uint32_t*>(buf + t0);
  const int64_t lim_g = n - t0;
  const int nsp = NS ? NS : sp.n;
#pragma unroll 1
  for (int k = 0; k < nsp; ++k) {
    const int s_k = sp.start[k], e_k = sp.end[k], w = e_k - s_k;
    const int sa = s_k < llen ? s_k : llen, sb = e_k < llen ? e_k : llen;
#if SCT_FQ_ABL == 5
    if (len) abl_sink(make_uint4((uint32_t)(sb - sa), (uint32_t)(k * to.cap + rec), 0u, 0u));
#else
    if (len) len[k * to.cap + rec] = sb - sa;
#endif
    if (!out) continue;
    const bool enc = SCT_FQ_ABL != 3 && k == 0 && is_seq && to.codes0 != nullptr;
    uint8_t* row0 = out + sp.prefix[k] * to.cap;
    uint8_t* o = row0 + rec * w;
    uint64_t code = 0;
    uint32_t fl = 0;
    const int s0 = start + sa;                    // the slice's tile offset
    const int wend = s0 + ((w + 15) & ~15) + 4;   // end of the last 16-byte window's dwords
    bool lut_row = false;
    if (sb - sa == w && sb <= clen && w > 0 && w <= 64 && wend <= lim_g) {
      const bool lds = wend <= lim_lds;
      const uintptr_t ob = (uintptr_t)row0;
      const int G = ((w | (int)ob) & 15) == 0 ? 16 : ((w | (int)ob) & 7) == 0 ? 8 : ((w | (int)ob) & 3) == 0 ? 4
                  : ((w | (int)ob) & 1) == 0 ? 2 : 1;
      for (int c = 0; c < w; c += 16) {
        const uint4 y = bytes16_at(tile32, gt, s0 + c, lds);
        const int m = w - c < 16 ? w - c : 16;
        store_row16(o + c, y, m, G);
        if (enc) {
          const uint32_t d[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (4 * j < m) enc_bases(d[j], m - 4 * j < 4 ? m - 4 * j : 4, to.code_kind, lut, code, fl);
        }
      }
    } else {
      const uint8_t* src = buf + t0 + start;
#pragma unroll 8
      for (int j = 0; j < w; ++j) {
        const int i = sa + j;
        o[j] = i < sb ? (i < clen ? src[i] : (uint8_t)'\n') : (uint8_t)0;
      }
      lut_row = enc;
    }
    if (lut_row) {  // span 0's row (as written, zero-padded) through the LUT
      code = 0;
      const uint8_t* src = buf + t0 + start;
      for (int j = 0; j < w; ++j) {
        const int i = sa + j;
        const uint8_t v = i < sb ? (i < clen ? src[i] : (uint8_t)'\n') : (uint8_t)0;
        const uint32_t en = lut[v];
        code = (code << to.code_kind) | (en & 7u);
        fl |= en;
      }
    }
#if SCT_FQ_ABL == 5
    if (enc) abl_sink(make_uint4((uint32_t)code, (uint32_t)(code >> 32), fl, (uint32_t)rec));
    continue;
#endif
    if (enc) {
      to.codes0[rec] = code;
      if (to.gc0) {
        const uint32_t g = (uint32_t)__popcll(code & to.gc_mask);
        to.gc0[rec] = (uint8_t)(g > 255 ? 255 : g);
      }
      if (to.flags0) to.flags0[rec] = (uint8_t)(((fl & F_AMBIG) ? 1u : 0u) | ((fl & F_INVALID) ? 2u : 0u));
    }
  }
}


__device__ __forceinline__ void tile_items(lds_u16* term, lds_u8* tile8, lds_u32* tile32, const uint8_t* lut,
                                           int ntile, int tmax, int64_t g0, int64_t t0, uint32_t nf, int head,
                                           const uint8_t* __restrict__ buf, int64_t n, Files fs, int text,
                                           const Spans& sp, const TileOut& to) {
  const int tid = threadIdx.x;
    // name lines: after terminators g = 3 (mod 4)
    for (int t = (int)((3 - (g0 & 3)) & 3) + 4 * tid; t < tmax; t += 4 * WG) {
      const uint32_t e = term[t];
      const int64_t o = (int64_t)(e & T16_OFF) + ((e & T16_VIRT) ? 0 : 1);  // the line's start in the tile
      const uint8_t ch = o < TILE + head ? tile8[o] : buf[t0 + o];
      if (ch != '@') atomicMax(to.d_status + 1, ~(unsigned long long)((g0 + t + 1) >> 2));
    }
    // sequence / quality lines: one item per line, its spans in turn; the first half of the
    // workgroup takes the sequence lines (after terminators t = -g0 mod 4), the second half the
    // quality lines (t = 2 - g0 mod 4), so every wave runs one kind (the CB encode is not carried
    // through the quality lines' waves)
    constexpr int HALF = WG / 2;
    // wave-uniform, and visibly so (readfirstlane): the row pointers and the store-width branches
    // of line_spans stay scalar
    const bool is_seq = __builtin_amdgcn_readfirstlane(tid) < HALF;
#if SCT_FQ_ABL == 2
    return;
#endif
    for (int t = (int)(((is_seq ? 0 : 2) - g0) & 3) + 4 * (tid & (HALF - 1)); t < tmax; t += 4 * HALF) {
      const int64_t line = g0 + t + 1, rec = line >> 2;
      if (rec >= to.cap) continue;
      const uint32_t e = term[t];
      const int start = (int)(e & T16_OFF) + ((e & T16_VIRT) ? 0 : 1);  // <= TILE
      int64_t cend;  // content end relative to the tile start
      int nl;
      if (t + 1 < (int)ntile) {  // the line ends at the tile's next terminator
        const uint32_t f = term[t + 1];
        cend = (int64_t)(f & T16_OFF) - ((f & T16_CRLF) ? 1 : 0);
        nl = (f & T16_VIRT) ? 0 : 1;
      } else if (nf != ~0u) {  // the tile's last line ends at the next tile's first terminator
        cend = TILE + (int64_t)(nf >> 2) - ((nf & 2u) ? 1 : 0);
        nl = (nf & 1u) ? 0 : 1;
      } else {  // the next tile's first terminator unknown: scan (max_end bytes, within its file)
        const int64_t next = t0 + start;
        int lo = 0, hi = fs.nfiles;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (fs.ends[mid] <= next) lo = mid + 1; else hi = mid;
        }
        const int64_t fe = lo < fs.nfiles ? fs.ends[lo] : n;
        const int64_t lim = next + sp.max_end < fe ? next + sp.max_end : fe;
        cend = lim - t0;
        nl = lim == fe ? 0 : 1;  // longer than the window: its end is irrelevant
        if (lim - t0 <= TILE + head) {  // inside the tile and the next tile's head staged after it
          for (int i = start; i < (int)(lim - t0); ++i) {
            const uint8_t ch = tile8[i];
            if (ch == '\n' || (text && ch == '\r')) {
              cend = i;
              nl = 1;
              break;
            }
          }
        } else {
          for (int64_t i = next; i < lim; ++i) {
            const uint8_t ch = buf[i];
            if (ch == '\n' || (text && ch == '\r')) {
              cend = i - t0;
              nl = 1;
              break;
            }
          }
        }
      }
      const int clen = (int)(cend - start), llen = clen + nl;  // < 2 TILE + max_end
      line_spans<0>(sp, to, is_seq, rec, start, clen, llen, tile32, lut, buf, n, t0, TILE + head);
    }
}

// Rows of records >= cap are skipped; span k's row r at out + cap * prefix_k + r * width_k, its
// length at len + k * cap + r; d_status[0] = the line count, d_status[1] = ~(first bad-name
// record) or 0 (records < lines / 4 only, as extract2_kernel); optionally span 0's sequence rows
// encoded as they are written (code_kind 2 TwoBit / 3 ThreeBit, one limb: width <= 32 / 21; gc
// and flags as sct_encode's).
__global__ __launch_bounds__(WG) void fastq_range_kernel(
    const uint8_t* __restrict__ buf, int64_t n, Files fs, int text, sct::TileSums ts,
    const uint32_t* __restrict__ first, int64_t ntiles, int64_t per_wg, int64_t cap, Spans sp,
    uint8_t* __restrict__ seq_out, uint8_t* __restrict__ qual_out, int32_t* __restrict__ seq_len,
    int32_t* __restrict__ qual_len, uint64_t* __restrict__ codes0, uint8_t* __restrict__ gc0,
    uint8_t* __restrict__ flags0, int code_kind, unsigned long long* __restrict__ d_status) {
  __shared__ uint16_t term[MAX_TERM];
  __shared__ uint4 tile_bytes[TILE / 16];
  __shared__ uint32_t w_cnt[WG / 64];
  __shared__ unsigned long long s_g0, s_total;
  __shared__ long long s_unused;
  __shared__ unsigned long long red[3][WG / 64];
  __shared__ uint8_t lut[256];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int64_t tile = (int64_t)blockIdx.x * per_wg;
  if (tile >= ntiles) return;  // (the whole workgroup)
  const int64_t tend = tile + per_wg < ntiles ? tile + per_wg : ntiles;
  if (codes0)
    for (int c = tid; c < 256; c += WG) lut[c] = lut_entry(code_kind, c);
  const TileOut to{seq_out, qual_out, seq_len, qual_len, codes0, gc0, flags0, code_kind,
                   code_kind == 2 ? 0x5555555555555555ull : 0x9249249249249249ull, cap, d_status};
  uint4 cur[SEG], nxt[SEG];
#pragma unroll
  for (int k = 0; k < SEG; ++k) cur[k] = load16(buf, n, tile * TILE + (int64_t)tid * TB + 16 * k);
  // (its barriers also cover the LUT)
  sct::tile_prefix<WG>(ts, tile, &s_g0, &s_unused, red, (ntiles + 1023) >> 10, &s_total);
  int64_t g0 = (int64_t)s_g0;  // global number of the current tile's first terminator
  const int64_t nrec = (int64_t)(s_total >> 2);
  const int64_t lim_g = 4 * nrec - 1;  // terminators beyond the last record's line 3 end nothing
  if (blockIdx.x == 0 && tid == 0) {
    d_status[0] = s_total;
    if (nrec > 0 && buf[0] != '@') atomicMax(d_status + 1, ~0ull);  // record 0's name line
  }
  uint32_t nf_cur = tile + 1 < ntiles ? first[tile + 1] : ~0u;
  FileCursor fc;
  // LDS-typed views of the tile (ds_read): a pointer that may be LDS or global compiles to flat
  // loads, after each of which the compiler waits for every load and store in flight
  lds_u8* tile8 = as_lds8(tile_bytes);
  lds_u32* tile32 = as_lds32(tile_bytes);
  for (; tile < tend; ++tile) {
    const int64_t ntl = tile + 1;
    const bool more = ntl < tend;
#pragma unroll
    for (int k = 0; k < SEG; ++k)
      nxt[k] = more ? load16(buf, n, ntl * TILE + (int64_t)tid * TB + 16 * k) : make_uint4(0, 0, 0, 0);
    const uint32_t nf_nxt = more && ntl + 1 < ntiles ? first[ntl + 1] : ~0u;
    const int64_t t0 = tile * TILE, p0 = t0 + (int64_t)tid * TB;
    const bool ends_here = fc.advance(fs, t0);
    Span spn{0, 0, 0, 0};
    if (p0 < n) spn = thread_span(buf, n, fs, text, p0, cur, ends_here);
    __syncthreads();  // the previous tile's readers of tile_bytes / term are done
#pragma unroll
    for (int k = 0; k < SEG; ++k) {
      tile_bytes[tid * SEG + k] = p0 + 16 * k < n ? cur[k] : make_uint4(0, 0, 0, 0);
      cur[k] = nxt[k];
    }
    const uint32_t tbits = spn.m | spn.vbits, c = __popc(tbits);
    uint32_t ic = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t x = __shfl_up(ic, d);
      if (lane >= d) ic += x;
    }
    if (lane == 63) w_cnt[wave] = ic;
    __syncthreads();
    uint32_t pre = ic - c, ntile = 0;
#pragma unroll
    for (int w = 0; w < WG / 64; ++w) {
      if (w < wave) pre += w_cnt[w];
      ntile += w_cnt[w];
    }
    {
      uint32_t bits = tbits, at = pre;
#if SCT_FQ_ABL == 4
      bits = 0;
#endif
      while (bits) {
        const int j = __ffs(bits) - 1;
        bits &= bits - 1;
        const uint32_t off = (uint32_t)(tid * TB + j);
        term[at++] = (spn.m >> j & 1u) ? (uint16_t)(off | ((spn.crlf >> j & 1u) ? T16_CRLF : 0u))
                                       : (uint16_t)((off + 1) | T16_VIRT);  // the file ends after byte off
      }
    }
    __syncthreads();
    const int tmax = (int)(g0 + ntile <= lim_g ? ntile : (lim_g > g0 ? lim_g - g0 : 0));
#if SCT_FQ_ABL != 1
    tile_items(as_lds16(term), tile8, tile32, lut, (int)ntile, tmax, g0, t0, nf_cur, 0, buf, n, fs, text, sp, to);
#endif
    g0 += ntile;
    nf_cur = nf_nxt;
  }
}

// grid of the persistent tile kernels: every resident workgroup slot once (at most ntiles)
unsigned resident_grid(const void* kernel, int64_t ntiles) {
  sct::scalar_quiesce();
  int dev = 0, cus = 256, per_cu = 0;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, WG, 0) != hipSuccess || per_cu <= 0) per_cu = 4;
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(ntiles, (int64_t)cus * per_cu));
}

// The byte just past line `target` (0-based line number; its terminator is terminator
// number `target` of the buffer): one workgroup finds the tile holding it (binary search of
// the tile offsets) and recounts that tile's terminators as extract2_kernel does.
__global__ __launch_bounds__(WG) void line_end_kernel(const uint8_t* __restrict__ buf, int64_t n, Files fs, int text,
                                                      const unsigned long long* __restrict__ offsets, int64_t ntiles,
                                                      unsigned long long target, long long* __restrict__ out) {
  int64_t lo = 0, hi = ntiles - 1;  // last tile k with offsets[k] <= target
  while (lo < hi) {
    const int64_t mid = (lo + hi + 1) >> 1;
    if (offsets[mid] <= target) lo = mid; else hi = mid - 1;
  }
  const int64_t t0 = lo * TILE, p0 = t0 + (int64_t)threadIdx.x * TB;
  uint32_t bits = 0;
  if (p0 < n) {
    uint4 v[SEG];
#pragma unroll
    for (int k = 0; k < SEG; ++k) v[k] = load16(buf, n, p0 + 16 * k);
    const Span sp = thread_span(buf, n, fs, text, p0, v, true);
    bits = sp.m | sp.vbits;
  }
  using BS = hipcub::BlockScan<uint32_t, WG>;
  __shared__ typename BS::TempStorage tmp;
  uint32_t pre;
  BS(tmp).ExclusiveSum((uint32_t)__popc(bits), pre);
  const unsigned long long want = target - offsets[lo];
  uint32_t at = pre;
  while (bits) {
    const int j = __ffs(bits) - 1;
    bits &= bits - 1;
    if (at == want) *out = p0 + j + 1;  // a real terminator ends at its byte; a virtual one at the file end
    ++at;
  }
}

}  // namespace

namespace {
// One spare index allocation per device, kept when an index is destroyed and taken by the
// next create that fits: a stream of pieces (one index per piece) or repeated extractions pay
// no hipMalloc / hipFree per call.  Every user of an index synchronises its stream before the
// index is destroyed (sct_fastq_extract_spans ends with one), so a cached or freed block is idle.
constexpr int kMaxDev = 16;
std::mutex g_ix_mu;
struct Spare {
  void* p = nullptr;
  size_t bytes = 0;
} g_ix_spare[kMaxDev];

hipError_t ix_alloc(void** p, size_t bytes, size_t* got) {
  int dev = 0;
  if (hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < kMaxDev) {
    std::lock_guard<std::mutex> g(g_ix_mu);
    Spare& sp = g_ix_spare[dev];
    if (sp.p && sp.bytes >= bytes) {
      *p = sp.p;
      *got = sp.bytes;
      sp.p = nullptr;
      sp.bytes = 0;
      return hipSuccess;
    }
  }
  *got = bytes;
  return hipMalloc(p, bytes);
}

void ix_release(void* p, size_t bytes) {
  if (!p) return;
  int dev = 0;
  if (hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < kMaxDev) {
    std::lock_guard<std::mutex> g(g_ix_mu);
    Spare& sp = g_ix_spare[dev];
    if (bytes > sp.bytes) {  // keep the larger block
      if (sp.p) (void)hipFree(sp.p);
      sp.p = p;
      sp.bytes = bytes;
      return;
    }
  }
  (void)hipFree(p);
}
}  // namespace

struct sct_fastq_index {
  int64_t nbytes = 0, nlines = 0, nrec = 0, first_bad = -2;
  int text = 0, nfiles = 0;
  int64_t ntiles = 0;
  void* d_mem = nullptr;                    // one allocation holding the arrays below
  size_t mem_bytes = 0;
  int64_t* d_ends = nullptr;                // file ends
  unsigned long long* d_offsets = nullptr;  // ntiles + 1 line offsets (exclusive scan of tile counts)
  uint32_t* d_first = nullptr;              // per tile: first terminator (see count_kernel)
  unsigned long long* d_bad = nullptr;      // first bad-name record of the last extraction
};

extern "C" int sct_fastq_index_destroy(sct_fastq_index* ix) {
  if (!ix) return SCT_OK;
  ix_release(ix->d_mem, ix->mem_bytes);
  delete ix;
  return SCT_OK;
}

extern "C" int sct_fastq_index_create(const uint8_t* d_buf, int64_t nbytes, const int64_t* file_ends,
                                      int nfiles, int text_mode, void* stream, sct_fastq_index** out) {
  SCT_CHECK(out != nullptr, "index is NULL");
  *out = nullptr;
  SCT_CHECK(nbytes >= 0 && (nbytes == 0 || d_buf != nullptr), "bad buffer");
  SCT_CHECK(nfiles >= 1 && file_ends != nullptr, "need at least one file end");
  for (int f = 0; f < nfiles; ++f)
    SCT_CHECK(file_ends[f] >= (f ? file_ends[f - 1] : 0) && file_ends[f] <= nbytes,
              "file_ends must be non-decreasing and <= nbytes");
  SCT_CHECK(file_ends[nfiles - 1] == nbytes, "the last file must end at nbytes");
  hipStream_t s = sct::as_stream(stream);
  auto* ix = new sct_fastq_index();
  auto fail_with = [&](int rc) {
    sct_fastq_index_destroy(ix);
    return rc;
  };
  ix->nbytes = nbytes;
  ix->text = text_mode ? 1 : 0;
  ix->nfiles = nfiles;
  ix->ntiles = std::max<int64_t>(1, sct::ceil_div(nbytes, TILE));
  SCT_CHECK(ix->ntiles < (1LL << 31), "buffer too large");
  // one allocation: ends | offsets | counts | first | flags, bad | scan scratch
  size_t tb = 0;
  SCT_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, (unsigned long long*)nullptr,
                                           (unsigned long long*)nullptr, (int)(ix->ntiles + 1), s));
  auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t o_ends = 0, o_off = up((size_t)nfiles * 8), o_cnt = o_off + up((ix->ntiles + 1) * 8),
               o_first = o_cnt + up((ix->ntiles + 1) * 8), o_flags = o_first + up(ix->ntiles * 4),
               o_tmp = o_flags + 256, total_bytes = o_tmp + up(tb);
  hipError_t e = ix_alloc(&ix->d_mem, total_bytes, &ix->mem_bytes);
  if (e != hipSuccess) return fail_with(sct::fail(SCT_E_NOMEM, "fastq index: %s", hipGetErrorString(e)));
  char* base = (char*)ix->d_mem;
  ix->d_ends = (int64_t*)(base + o_ends);
  ix->d_offsets = (unsigned long long*)(base + o_off);
  ix->d_first = (uint32_t*)(base + o_first);
  unsigned long long* d_counts = (unsigned long long*)(base + o_cnt);
  unsigned* d_flags = (unsigned*)(base + o_flags);
  ix->d_bad = (unsigned long long*)(base + o_flags + 8);
  void* d_tmp = base + o_tmp;
  SCT_HIP(hipMemcpyAsync(ix->d_ends, file_ends, (size_t)nfiles * 8, hipMemcpyHostToDevice, s));
  SCT_HIP(hipMemsetAsync(d_flags, 0, 8, s));
  SCT_HIP(hipMemsetAsync(d_counts, 0, (size_t)(ix->ntiles + 1) * 8, s));
  const Files fs{ix->d_ends, nfiles};
  if (nbytes > 0)
    hipLaunchKernelGGL(count_kernel, dim3(resident_grid((const void*)count_kernel, ix->ntiles)), dim3(WG), 0, s,
                       d_buf, nbytes, fs, ix->text, d_counts, ix->d_first, d_flags, ix->ntiles);
  SCT_LAUNCH_CHECK();
  SCT_HIP(hipcub::DeviceScan::ExclusiveSum(d_tmp, tb, d_counts, ix->d_offsets, (int)(ix->ntiles + 1), s));
  unsigned long long total = 0;
  unsigned flags = 0;
  SCT_HIP(hipMemcpyAsync(&total, ix->d_offsets + ix->ntiles, 8, hipMemcpyDeviceToHost, s));
  SCT_HIP(hipMemcpyAsync(&flags, d_flags, 4, hipMemcpyDeviceToHost, s));
  SCT_HIP(hipStreamSynchronize(s));
  if (ix->text && (flags & 1u))
    return fail_with(sct::fail(SCT_E_RANGE, "text-mode FASTQ must be ASCII on the device path "
                                            "(read it in 'rb' mode)"));
  ix->nlines = (int64_t)total;
  ix->nrec = (int64_t)total / 4;
  *out = ix;
  return SCT_OK;
}

extern "C" int sct_fastq_index_info(const sct_fastq_index* ix, int64_t* nrecords, int64_t* nlines,
                                    int64_t* first_bad_name) {
  SCT_CHECK(ix != nullptr, "index is NULL");
  if (nrecords) *nrecords = ix->nrec;
  if (nlines) *nlines = ix->nlines;
  if (first_bad_name) *first_bad_name = ix->first_bad;
  return SCT_OK;
}

extern "C" int sct_fastq_extract_spans(sct_fastq_index* ix, const uint8_t* d_buf, const int32_t* spans,
                                       int nspans, uint8_t* d_seq, uint8_t* d_qual, int32_t* d_seq_len,
                                       int32_t* d_qual_len, int64_t* first_bad_name, void* stream) {
  SCT_CHECK(ix != nullptr, "index is NULL");
  SCT_CHECK(nspans >= 0 && nspans <= MAX_SPANS && (nspans == 0 || spans), "0..%d spans", MAX_SPANS);
  Spans sp{};
  sp.n = nspans;
  int64_t pre = 0;
  for (int k = 0; k < nspans; ++k) {
    SCT_CHECK(0 <= spans[2 * k] && spans[2 * k] <= spans[2 * k + 1] && spans[2 * k + 1] <= 4096,
              "span %d = [%d, %d) unsupported", k, spans[2 * k], spans[2 * k + 1]);
    sp.start[k] = spans[2 * k];
    sp.end[k] = spans[2 * k + 1];
    sp.prefix[k] = pre;
    sp.max_end = std::max(sp.max_end, sp.end[k]);
    pre += sp.end[k] - sp.start[k];
  }
  sp.width = (int)pre;
  hipStream_t s = sct::as_stream(stream);
  SCT_HIP(hipMemsetAsync(ix->d_bad, 0xFF, 8, s));
  if (ix->nbytes > 0) {
    SCT_CHECK(d_buf != nullptr, "buffer is NULL");
    const Files fs{ix->d_ends, ix->nfiles};
    hipLaunchKernelGGL(extract2_kernel, dim3(resident_grid((const void*)extract2_kernel, ix->ntiles)), dim3(WG), 0, s,
                       d_buf, ix->nbytes, fs,
                       ix->text, ix->d_offsets, ix->d_first, ix->ntiles, ix->nrec, sp, d_seq, d_qual,
                       d_seq_len, d_qual_len, ix->d_bad);
    SCT_LAUNCH_CHECK();
  }
  unsigned long long bad = ~0ull;
  SCT_HIP(hipMemcpyAsync(&bad, ix->d_bad, 8, hipMemcpyDeviceToHost, s));
  SCT_HIP(hipStreamSynchronize(s));
  ix->first_bad = bad == ~0ull ? -1 : (int64_t)bad;
  if (first_bad_name) *first_bad_name = ix->first_bad;
  return SCT_OK;
}

namespace {
#define SCT_TRY(x)                 \
  do {                             \
    int rc_ = (x);                 \
    if (rc_ != SCT_OK) return rc_; \
  } while (0)
}  // namespace

// Extraction without an index (fq_count_kernel, tile_sums_reduce_kernel, fastq_range_kernel),
// asynchronous on `stream`: the concatenated files in d_buf, their cumulative ends in d_file_ends
// (DEVICE memory, nfiles entries, the last = nbytes).  Rows are laid out by cap_records (span
// k's row r at out + cap * prefix_k + r * width_k, its length at len + k * cap + r; rows of
// records >= cap_records are not written); d_status (3 x int64, device) receives the line count
// (records = lines / 4), ~(first bad-name record) or 0, and a text-mode non-ASCII flag.
// d_codes0 / d_gc0 / d_flags0 (nullable): span 0's sequence rows encoded (code_kind 2 TwoBit,
// width <= 32; 3 ThreeBit, width <= 21: N kept as 6, the input of sct_nearest_query).
extern "C" int sct_fastq_extract_fused(const uint8_t* d_buf, int64_t nbytes, const int64_t* d_file_ends, int nfiles,
                                       int text_mode, const int32_t* spans, int nspans, int64_t cap_records,
                                       uint8_t* d_seq, uint8_t* d_qual, int32_t* d_seq_len, int32_t* d_qual_len,
                                       uint64_t* d_codes0, uint8_t* d_gc0, uint8_t* d_flags0, int code_kind,
                                       int64_t* d_status, void* stream) {
  SCT_CHECK(d_status != nullptr && nfiles >= 1 && d_file_ends != nullptr, "bad arguments");
  SCT_CHECK(nbytes >= 0 && (nbytes == 0 || d_buf != nullptr) && cap_records >= 0, "bad buffer");
  SCT_CHECK(nspans >= 0 && nspans <= MAX_SPANS && (nspans == 0 || spans), "0..%d spans", MAX_SPANS);
  Spans sp{};
  sp.n = nspans;
  int64_t pre = 0;
  for (int k = 0; k < nspans; ++k) {
    SCT_CHECK(0 <= spans[2 * k] && spans[2 * k] <= spans[2 * k + 1] && spans[2 * k + 1] <= 4096,
              "span %d = [%d, %d) unsupported", k, spans[2 * k], spans[2 * k + 1]);
    sp.start[k] = spans[2 * k];
    sp.end[k] = spans[2 * k + 1];
    sp.prefix[k] = pre;
    sp.max_end = std::max(sp.max_end, sp.end[k]);
    pre += sp.end[k] - sp.start[k];
  }
  sp.width = (int)pre;
  SCT_CHECK(code_kind == 2 || code_kind == 3, "code_kind must be 2 or 3");
  SCT_CHECK(!d_codes0 || (nspans >= 1 && code_kind * (sp.end[0] - sp.start[0]) <= 64 && d_seq),
            "span 0 encode needs one limb (width <= %d)", 64 / code_kind);
  hipStream_t s = sct::as_stream(stream);
  SCT_HIP(hipMemsetAsync(d_status, 0, 24, s));
  if (nbytes == 0) return SCT_OK;
  const int64_t ntiles = sct::ceil_div(nbytes, TILE);
  // fq_count_kernel runs one workgroup per tile and a launch holds < 2^32 threads
  SCT_CHECK(ntiles * WG < (1LL << 32), "buffer too large: %lld bytes (one launch covers < %lld bytes; pass the "
            "files in pieces, sct_fastq_stream_*)", (long long)nbytes, (long long)(((1LL << 32) / WG) * TILE));
  void* scratch = nullptr;
  const size_t sbytes = sct::tile_sums_bytes(ntiles), fbytes = (size_t)ntiles * 4;
  SCT_HIP(sct::pool_alloc(&scratch, sbytes + fbytes, s));
  const sct::TileSums ts = sct::tile_sums_at(scratch, ntiles, false);
  uint32_t* first = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(scratch) + sbytes);
  const Files fs{d_file_ends, nfiles};
  hipLaunchKernelGGL(fq_count_kernel, dim3((unsigned)ntiles), dim3(WG), 0, s, d_buf, nbytes, fs, text_mode ? 1 : 0, ts,
                     first, reinterpret_cast<unsigned*>(d_status + 2));
  hipLaunchKernelGGL(sct::tile_sums_reduce_kernel, dim3((unsigned)sct::ceil_div(ntiles, 1024)), dim3(64), 0, s, ts,
                     ntiles);
  // contiguous tile ranges, one per resident workgroup slot
  // contiguous ranges of 8 tiles (64 KiB) per workgroup: 1.09-1.10 ms per 20M records against
  // 1.13-1.20 for one range per resident slot and 1.55 for one tile per workgroup (same box,
  // tools/ingest_tiles_ab.py); SCT_TUNE_INGEST_TILES = 0 sizes the ranges to the resident grid
  const int64_t knob = sct::tune(SCT_TUNE_INGEST_TILES, -1);
  const int64_t per_wg = knob > 0   ? knob
                         : knob < 0 ? 8
                                    : sct::ceil_div(ntiles, (int64_t)resident_grid((const void*)fastq_range_kernel, ntiles));
  hipLaunchKernelGGL(fastq_range_kernel, dim3((unsigned)sct::ceil_div(ntiles, per_wg)), dim3(WG), 0, s, d_buf, nbytes,
                     fs, text_mode ? 1 : 0, ts, (const uint32_t*)first, ntiles, per_wg, cap_records, sp, d_seq, d_qual,
                     d_seq_len, d_qual_len, d_codes0, d_gc0, d_flags0, code_kind,
                     reinterpret_cast<unsigned long long*>(d_status));
  hipError_t e = hipGetLastError();
  sct::pool_free(scratch, s);
  if (e != hipSuccess) return sct::fail(SCT_E_HIP, "fastq fused: %s", hipGetErrorString(e));
  return SCT_OK;
}

extern "C" int sct_fastq_extract_host(const uint8_t* buf, int64_t nbytes, const int64_t* file_ends,
                                      int nfiles, int text_mode, const int32_t* spans, int nspans,
                                      uint8_t* seq_out, uint8_t* qual_out, int32_t* seq_len,
                                      int32_t* qual_len, int64_t max_records, int64_t* nrecords,
                                      int64_t* first_bad_name) {
  SCT_CHECK(nrecords != nullptr, "nrecords is NULL");
  SCT_CHECK(nspans >= 0 && (nspans == 0 || spans != nullptr), "bad spans");
  sct::DevBuf d_buf;
  SCT_HIP(d_buf.alloc((size_t)nbytes));
  if (nbytes) SCT_HIP(hipMemcpy(d_buf.p, buf, (size_t)nbytes, hipMemcpyHostToDevice));
  sct_fastq_index* ix = nullptr;
  SCT_TRY(sct_fastq_index_create((const uint8_t*)d_buf.p, nbytes, file_ends, nfiles, text_mode, nullptr, &ix));
  struct Guard {
    sct_fastq_index* p;
    ~Guard() { sct_fastq_index_destroy(p); }
  } g{ix};
  *nrecords = ix->nrec;
  if (max_records < ix->nrec) return SCT_OK;  // sizing call: outputs untouched
  // spans laid out back to back: row r of span k at out + nrec * off_k + r * width_k
  int64_t width = 0;
  for (int k = 0; k < nspans; ++k) width += (int64_t)spans[2 * k + 1] - spans[2 * k];
  const int64_t bytes = width * ix->nrec;
  const size_t lbytes = (size_t)ix->nrec * nspans * 4;
  sct::DevBuf d_s, d_q, d_sl, d_ql;
  SCT_HIP(d_s.alloc((size_t)bytes));
  SCT_HIP(d_q.alloc((size_t)bytes));
  SCT_HIP(d_sl.alloc(lbytes));
  SCT_HIP(d_ql.alloc(lbytes));
  SCT_TRY(sct_fastq_extract_spans(ix, (const uint8_t*)d_buf.p, spans, nspans,
                                  seq_out ? (uint8_t*)d_s.p : nullptr, qual_out ? (uint8_t*)d_q.p : nullptr,
                                  seq_len ? (int32_t*)d_sl.p : nullptr, qual_len ? (int32_t*)d_ql.p : nullptr,
                                  first_bad_name, nullptr));
  if (seq_out && bytes) SCT_HIP(hipMemcpy(seq_out, d_s.p, (size_t)bytes, hipMemcpyDeviceToHost));
  if (qual_out && bytes) SCT_HIP(hipMemcpy(qual_out, d_q.p, (size_t)bytes, hipMemcpyDeviceToHost));
  if (seq_len && lbytes) SCT_HIP(hipMemcpy(seq_len, d_sl.p, lbytes, hipMemcpyDeviceToHost));
  if (qual_len && lbytes) SCT_HIP(hipMemcpy(qual_len, d_ql.p, lbytes, hipMemcpyDeviceToHost));
  return SCT_OK;
}

// ---------------------------------------------------------------- streaming (chunked) ingest
// reader.Reader iterates its files lazily (src/sctools/reader.py:56-85); a FASTQ stream of
// a billion reads never sits in host memory whole.  A stream object keeps its device
// buffers across chunks: the caller passes consecutive pieces of the concatenated files
// (each ending on a '\n' unless it is the last), every complete record of a piece is
// extracted, and `consumed` says where the next piece must start (the lines of a record
// cut by the piece end are carried over by the caller).
struct sct_fastq_stream {
  int text = 0, nspans = 0, qualities = 1;
  int32_t spans[2 * MAX_SPANS] = {};
  int64_t width = 0;  // sum of span widths
  sct::HostStage* st = nullptr;
  void* d_buf = nullptr;
  int64_t buf_cap = 0;
  void* d_out = nullptr;  // seq | qual | seq_len | qual_len for rec_cap records
  int64_t rec_cap = 0;
  long long* d_end = nullptr;
  int64_t nrec = 0, first_bad = -1, consumed = 0;
  // the next piece copied ahead (sct_fastq_stream_stage): into d_next on copy_stream, `staged`
  // recorded after it; the chunk call for (staged_ptr, staged_n) swaps d_next in
  void* d_next = nullptr;
  int64_t next_cap = 0;
  hipStream_t copy_stream = nullptr;
  hipEvent_t staged = nullptr;
  const uint8_t* staged_ptr = nullptr;
  int64_t staged_n = -1;
};

extern "C" int sct_fastq_stream_destroy(sct_fastq_stream* s) {
  if (!s) return SCT_OK;
  if (s->copy_stream) {
    (void)hipStreamSynchronize(s->copy_stream);
    (void)hipStreamDestroy(s->copy_stream);
  }
  if (s->staged) (void)hipEventDestroy(s->staged);
  if (s->d_next) (void)hipFree(s->d_next);
  if (s->st) (void)hipStreamSynchronize(s->st->stream);  // nothing of the stream's still reads its buffers
  if (s->d_buf) (void)hipFree(s->d_buf);
  if (s->d_out) (void)hipFree(s->d_out);
  if (s->d_end) (void)hipFree(s->d_end);
  delete s;
  return SCT_OK;
}

extern "C" int sct_fastq_stream_create(int text_mode, const int32_t* spans, int nspans, int qualities,
                                       sct_fastq_stream** out) {
  SCT_CHECK(out != nullptr, "stream is NULL");
  *out = nullptr;
  SCT_CHECK(nspans >= 0 && nspans <= MAX_SPANS && (nspans == 0 || spans), "0..%d spans", MAX_SPANS);
  auto* s = new sct_fastq_stream();
  s->text = text_mode ? 1 : 0;
  s->nspans = nspans;
  s->qualities = qualities ? 1 : 0;
  for (int k = 0; k < nspans; ++k) {
    if (!(0 <= spans[2 * k] && spans[2 * k] <= spans[2 * k + 1] && spans[2 * k + 1] <= 4096)) {
      delete s;
      return sct::fail(SCT_E_INVALID, "span %d = [%d, %d) unsupported", k, spans[2 * k], spans[2 * k + 1]);
    }
    s->spans[2 * k] = spans[2 * k];
    s->spans[2 * k + 1] = spans[2 * k + 1];
    s->width += spans[2 * k + 1] - spans[2 * k];
  }
  s->st = sct::host_stage();
  if (!s->st || hipMalloc((void**)&s->d_end, 8) != hipSuccess) {
    sct_fastq_stream_destroy(s);
    return sct::fail(SCT_E_HIP, "fastq stream: device setup failed");
  }
  *out = s;
  return SCT_OK;
}

// One piece: extract its complete records on the device.  final = 0: `consumed` = the byte
// just past the last complete record; final = 1: the whole piece is consumed (a trailing
// incomplete record is dropped, as the reference's grouper drops it).
extern "C" int sct_fastq_stream_chunk(sct_fastq_stream* s, const uint8_t* buf, int64_t nbytes,
                                      const int64_t* file_ends, int nfiles, int final, int64_t* nrecords,
                                      int64_t* consumed, int64_t* first_bad_name) {
  SCT_CHECK(s && nrecords && consumed && first_bad_name, "NULL pointer");
  SCT_CHECK(nbytes >= 0 && (nbytes == 0 || buf), "bad buffer");
  hipStream_t hs = s->st->stream;
  const bool was_staged = s->staged_n >= 0 && s->staged_ptr == buf && s->staged_n == nbytes;
  if (s->staged_n >= 0) {  // (a staged copy is complete before anything else touches its buffers)
    SCT_HIP(hipStreamWaitEvent(hs, s->staged, 0));
    s->staged_n = -1;
    s->staged_ptr = nullptr;
    if (was_staged) {  // the piece is on the device already: its buffer becomes this chunk's
      std::swap(s->d_buf, s->d_next);
      std::swap(s->buf_cap, s->next_cap);
    }
  }
  if (nbytes > s->buf_cap) {
    if (s->d_buf) (void)hipFree(s->d_buf);
    s->d_buf = nullptr;
    s->buf_cap = 0;
    SCT_HIP(hipMalloc(&s->d_buf, (size_t)nbytes));
    s->buf_cap = nbytes;
  }
  if (was_staged) {
    // (copied by sct_fastq_stream_stage)
  } else if (sct::host_range_pinned(buf, (size_t)nbytes)) {
    // a page-locked piece (the Python layer reads the files into one): one DMA in place; the
    // call returns only after a synchronisation of `hs`, so the caller may refill it afterwards
    if (nbytes) SCT_HIP(hipMemcpyAsync(s->d_buf, buf, (size_t)nbytes, hipMemcpyHostToDevice, hs));
  } else {
    // through the stage's pinned buffer in 64 MB pieces: page-locked copies, no per-call pinning
    constexpr size_t kPiece = 64ull << 20;
    SCT_TRY(sct::stage_reserve(s->st, std::min<size_t>((size_t)nbytes, kPiece), 0));
    for (int64_t o = 0; o < nbytes; o += (int64_t)kPiece) {
      const size_t len = (size_t)std::min<int64_t>((int64_t)kPiece, nbytes - o);
      SCT_HIP(hipStreamSynchronize(hs));  // the previous piece's copy has left the pinned buffer
      memcpy(s->st->pinned, buf + o, len);
      SCT_HIP(hipMemcpyAsync((uint8_t*)s->d_buf + o, s->st->pinned, len, hipMemcpyHostToDevice, hs));
    }
  }
  sct_fastq_index* ix = nullptr;
  SCT_TRY(sct_fastq_index_create((const uint8_t*)s->d_buf, nbytes, file_ends, nfiles, s->text, hs, &ix));
  struct Guard {
    sct_fastq_index* p;
    ~Guard() { sct_fastq_index_destroy(p); }
  } g{ix};
  const int64_t nrec = ix->nrec;
  if (nrec > s->rec_cap) {
    if (s->d_out) (void)hipFree(s->d_out);
    s->d_out = nullptr;
    s->rec_cap = 0;
    const int64_t cap = nrec + nrec / 4 + 1024;
    SCT_HIP(hipMalloc(&s->d_out, (size_t)cap * (2 * s->width + 8 * s->nspans) + 256));
    s->rec_cap = cap;
  }
  uint8_t* d_seq = (uint8_t*)s->d_out;
  uint8_t* d_qual = d_seq + s->rec_cap * s->width;
  int32_t* d_sl = (int32_t*)(d_qual + s->rec_cap * s->width);
  int32_t* d_ql = d_sl + s->rec_cap * s->nspans;
  int64_t bad = -1;
  SCT_TRY(sct_fastq_extract_spans(ix, (const uint8_t*)s->d_buf, s->spans, s->nspans, d_seq,
                                  s->qualities ? d_qual : nullptr, d_sl, s->qualities ? d_ql : nullptr, &bad, hs));
  int64_t used = nbytes;
  if (!final) {
    used = 0;
    if (nrec > 0) {
      hipLaunchKernelGGL(line_end_kernel, dim3(1), dim3(WG), 0, hs, (const uint8_t*)s->d_buf, nbytes,
                         Files{ix->d_ends, ix->nfiles}, s->text, ix->d_offsets, ix->ntiles,
                         (unsigned long long)(4 * nrec - 1), s->d_end);
      SCT_LAUNCH_CHECK();
      long long e = -1;
      SCT_HIP(hipMemcpyAsync(&e, s->d_end, 8, hipMemcpyDeviceToHost, hs));
      SCT_HIP(hipStreamSynchronize(hs));
      SCT_CHECK(e > 0 && e <= nbytes, "record end not found");
      used = e;
    }
  }
  if (final) SCT_HIP(hipStreamSynchronize(hs));  // (the piece's buffer is the caller's again)
  s->nrec = nrec;
  s->first_bad = bad;
  s->consumed = used;
  *nrecords = nrec;
  *consumed = used;
  *first_bad_name = bad;
  return SCT_OK;
}

extern "C" int sct_fastq_stream_stage(sct_fastq_stream* s, const uint8_t* buf, int64_t nbytes) {
  SCT_CHECK(s != nullptr, "stream is NULL");
  SCT_CHECK(nbytes >= 0 && (nbytes == 0 || buf), "bad buffer");
  if (s->staged_n >= 0) {  // a previous stage never used: its copy must end before d_next is reused
    SCT_HIP(hipEventSynchronize(s->staged));
    s->staged_n = -1;
    s->staged_ptr = nullptr;
  }
  if (nbytes == 0 || !sct::host_range_pinned(buf, (size_t)nbytes)) return SCT_OK;  // (the chunk call copies)
  if (!s->copy_stream) SCT_HIP(hipStreamCreateWithFlags(&s->copy_stream, hipStreamNonBlocking));
  if (!s->staged) SCT_HIP(hipEventCreateWithFlags(&s->staged, hipEventDisableTiming));
  if (nbytes > s->next_cap) {
    if (s->d_next) {
      SCT_HIP(hipStreamSynchronize(s->st->stream));  // (no chunk kernel reads the old buffer)
      (void)hipFree(s->d_next);
    }
    s->d_next = nullptr;
    s->next_cap = 0;
    SCT_HIP(hipMalloc(&s->d_next, (size_t)nbytes));
    s->next_cap = nbytes;
  }
  // d_next was the previous chunk's buffer two pieces ago at most: the copy waits for the chunk
  // work queued so far on the stream (its index and extraction read d_buf, not d_next, but a
  // swapped-out buffer may still be read by the last chunk's kernels)
  SCT_HIP(hipEventRecord(s->staged, s->st->stream));
  SCT_HIP(hipStreamWaitEvent(s->copy_stream, s->staged, 0));
  SCT_HIP(hipMemcpyAsync(s->d_next, buf, (size_t)nbytes, hipMemcpyHostToDevice, s->copy_stream));
  SCT_HIP(hipEventRecord(s->staged, s->copy_stream));
  s->staged_ptr = buf;
  s->staged_n = nbytes;
  return SCT_OK;
}

// The last piece's outputs, laid out as sct_fastq_extract_host's (nullable each).
extern "C" int sct_fastq_stream_fetch(sct_fastq_stream* s, uint8_t* seq_out, uint8_t* qual_out, int32_t* seq_len,
                                      int32_t* qual_len) {
  SCT_CHECK(s != nullptr, "stream is NULL");
  SCT_CHECK(s->qualities || (!qual_out && !qual_len), "stream created without qualities");
  hipStream_t hs = s->st->stream;
  const int64_t n = s->nrec;
  if (n == 0) return SCT_OK;
  const uint8_t* d_seq = (const uint8_t*)s->d_out;
  const uint8_t* d_qual = d_seq + s->rec_cap * s->width;
  const int32_t* d_sl = (const int32_t*)(d_qual + s->rec_cap * s->width);
  const int32_t* d_ql = d_sl + s->rec_cap * s->nspans;
  // the extraction lays span k's rows out at n * prefix_k and its lengths at n * k, as here
  if (seq_out && s->width) SCT_HIP(hipMemcpyAsync(seq_out, d_seq, (size_t)(n * s->width), hipMemcpyDeviceToHost, hs));
  if (qual_out && s->width)
    SCT_HIP(hipMemcpyAsync(qual_out, d_qual, (size_t)(n * s->width), hipMemcpyDeviceToHost, hs));
  if (seq_len && s->nspans)
    SCT_HIP(hipMemcpyAsync(seq_len, d_sl, (size_t)n * s->nspans * 4, hipMemcpyDeviceToHost, hs));
  if (qual_len && s->nspans)
    SCT_HIP(hipMemcpyAsync(qual_len, d_ql, (size_t)n * s->nspans * 4, hipMemcpyDeviceToHost, hs));
  SCT_HIP(hipStreamSynchronize(hs));
  return SCT_OK;
}
