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
// Two passes over 4 KiB tiles (16 bytes per thread, SWAR '\n' compares): count each tile's
// line ends, exclusive-scan them into every tile's first line number, then store every end
// as the next line's start; the lengths follow from consecutive starts.  The
// variable-length TwoBit/ThreeBit encoder (sct_encode_var) packs the lines straight from
// the file bytes.
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "sct_common.h"

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
  SCT_CHECK(ntiles < (1LL << 31), "buffer too large");
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
  sct::DevBuf d_buf;
  SCT_HIP(d_buf.alloc((size_t)nbytes));
  if (nbytes) SCT_HIP(hipMemcpyAsync(d_buf.p, buf, (size_t)nbytes, hipMemcpyHostToDevice, st->stream));
  int64_t n = 0;
  int rc = sct_lines((const uint8_t*)d_buf.p, nbytes, 0, nullptr, nullptr, &n, max_len, st->stream);
  if (rc != SCT_OK) return rc;
  *nlines = n;
  if (max_lines < n || n == 0) {
    if (n == 0) *max_len = 0;
    if (max_lines < n) {  // the sizing call also needs the longest line
      sct::DevBuf s0, l0;
      SCT_HIP(s0.alloc((size_t)n * 8));
      SCT_HIP(l0.alloc((size_t)n * 4));
      int64_t n2 = 0;
      rc = sct_lines((const uint8_t*)d_buf.p, nbytes, n, (int64_t*)s0.p, (int32_t*)l0.p, &n2, max_len, st->stream);
      if (rc != SCT_OK) return rc;
    }
    return SCT_OK;
  }
  SCT_CHECK(codes && starts && lens && flags, "NULL output");
  sct::DevBuf ds, dl, dc, df;
  SCT_HIP(ds.alloc((size_t)n * 8));
  SCT_HIP(dl.alloc((size_t)n * 4));
  SCT_HIP(dc.alloc((size_t)n * words * 8));
  SCT_HIP(df.alloc((size_t)n));
  int64_t n2 = 0;
  rc = sct_lines((const uint8_t*)d_buf.p, nbytes, n, (int64_t*)ds.p, (int32_t*)dl.p, &n2, max_len, st->stream);
  if (rc != SCT_OK) return rc;
  SCT_CHECK((int64_t)kind * *max_len <= (int64_t)words * 64, "words %d too few for lines of %d bases", words,
            *max_len);
  rc = sct_encode_var(kind, (const uint8_t*)d_buf.p, (const int64_t*)ds.p, (const int32_t*)dl.p, n, words,
                      (uint64_t*)dc.p, nullptr, (uint8_t*)df.p, st->stream);
  if (rc != SCT_OK) return rc;
  SCT_HIP(hipMemcpyAsync(codes, dc.p, (size_t)n * words * 8, hipMemcpyDeviceToHost, st->stream));
  SCT_HIP(hipMemcpyAsync(starts, ds.p, (size_t)n * 8, hipMemcpyDeviceToHost, st->stream));
  SCT_HIP(hipMemcpyAsync(lens, dl.p, (size_t)n * 4, hipMemcpyDeviceToHost, st->stream));
  SCT_HIP(hipMemcpyAsync(flags, df.p, (size_t)n, hipMemcpyDeviceToHost, st->stream));
  SCT_HIP(hipStreamSynchronize(st->stream));
  return SCT_OK;
}
