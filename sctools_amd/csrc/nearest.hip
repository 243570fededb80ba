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
// one block.  For each block the whitelist is bucketed by that block's bits (CSR:
// offsets[key] .. offsets[key+1] into (code, index) arrays, built by a histogram /
// exclusive-scan / scatter on the GPU); a query probes its P buckets and verifies every
// candidate with the full distance, so false candidates (and 24-bit key truncation for
// very wide blocks) never change the result.  A code found through several blocks has
// one index, so it is never counted as a tie with itself.
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "sct_common.h"

namespace {

constexpr int WG = 256;
constexpr int MAX_PARTS = 8;
constexpr int KEY_BITS_MAX = 24;

struct Part {
  int lo_bit;    // first bit of the block in the code
  int nbits;     // bits of the block
  int key_bits;  // min(nbits, 24): keys are the block's low key_bits bits
};

__device__ __forceinline__ uint32_t part_key(uint64_t code, Part p) {
  return (uint32_t)((code >> p.lo_bit) & ((1ull << p.key_bits) - 1ull));
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
    atomicAdd(&counts[part_key(wl[j], part)], 1u);
}

__global__ void key_scatter_kernel(const uint64_t* __restrict__ wl, int64_t nw, Part part,
                                   uint32_t* __restrict__ cursor, uint64_t* __restrict__ b_codes,
                                   int32_t* __restrict__ b_index) {
  for (int64_t j = (int64_t)blockIdx.x * WG + threadIdx.x; j < nw; j += (int64_t)gridDim.x * WG) {
    const uint64_t w = wl[j];
    const uint32_t pos = atomicAdd(&cursor[part_key(w, part)], 1u);
    b_codes[pos] = w;
    b_index[pos] = (int32_t)j;
  }
}

template <int KIND>
__global__ __launch_bounds__(WG) void nearest_query_kernel(
    const uint64_t* __restrict__ queries, int64_t nq, int nparts, Parts parts,
    const uint32_t* const* __restrict__ offsets, const uint64_t* const* __restrict__ b_codes,
    const int32_t* const* __restrict__ b_index, int max_d, int32_t* __restrict__ out_index,
    uint8_t* __restrict__ out_dist) {
  for (int64_t i = (int64_t)blockIdx.x * WG + threadIdx.x; i < nq; i += (int64_t)gridDim.x * WG) {
    const uint64_t q = queries[i];
    int best_d = max_d + 1, best_j = -1;
    bool tie = false;
    for (int p = 0; p < nparts; ++p) {
      const uint32_t key = part_key(q, parts.p[p]);
      const uint32_t* off = offsets[p];
      const uint32_t lo = off[key], hi = off[key + 1];
      const uint64_t* bc = b_codes[p];
      const int32_t* bi = b_index[p];
      for (uint32_t t = lo; t < hi; ++t) {
        const int d = KIND == 2 ? dist2(q, bc[t]) : dist3(q, bc[t]);
        if (d < best_d) {
          best_d = d;
          best_j = bi[t];
          tie = false;
        } else if (d == best_d) {
          const int j = bi[t];
          if (j != best_j) tie = true;
        }
      }
    }
    out_index[i] = best_j < 0 ? -1 : (tie ? -2 : best_j);
    out_dist[i] = best_j < 0 ? (uint8_t)255 : (uint8_t)best_d;
  }
}

unsigned grid_for(int64_t n, int64_t cap = 16384) {
  const int64_t b = sct::ceil_div(n, WG);
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(b, cap));
}

}  // namespace

struct sct_nearest_plan {
  int kind = 2, max_d = 0, nparts = 0, code_bits = 0;
  int64_t nw = 0;
  Parts parts{};
  uint32_t* d_offsets[MAX_PARTS] = {};
  uint64_t* d_bcodes[MAX_PARTS] = {};
  int32_t* d_bindex[MAX_PARTS] = {};
  // device copies of the pointer tables above
  const uint32_t** d_off_tab = nullptr;
  const uint64_t** d_code_tab = nullptr;
  const int32_t** d_idx_tab = nullptr;
};

extern "C" int sct_nearest_plan_destroy(sct_nearest_plan* p) {
  if (!p) return SCT_OK;
  for (int k = 0; k < MAX_PARTS; ++k) {
    if (p->d_offsets[k]) (void)hipFree(p->d_offsets[k]);
    if (p->d_bcodes[k]) (void)hipFree(p->d_bcodes[k]);
    if (p->d_bindex[k]) (void)hipFree(p->d_bindex[k]);
  }
  if (p->d_off_tab) (void)hipFree(p->d_off_tab);
  if (p->d_code_tab) (void)hipFree(p->d_code_tab);
  if (p->d_idx_tab) (void)hipFree(p->d_idx_tab);
  delete p;
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
  for (int k = 0; k < p->nparts; ++k) {
    const int pos_lo = G * k / p->nparts, pos_hi = G * (k + 1) / p->nparts;
    Part& pt = p->parts.p[k];
    pt.lo_bit = pos_lo * kind;
    pt.nbits = std::min(64, pos_hi * kind) - pt.lo_bit;
    pt.key_bits = std::min(pt.nbits, KEY_BITS_MAX);
  }
  size_t scan_bytes = 0;
  for (int k = 0; k < p->nparts; ++k) {
    size_t b = 0;
    const int nkeys = 1 << p->parts.p[k].key_bits;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, b, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                           nkeys + 1, s);
    scan_bytes = std::max(scan_bytes, b);
  }
  sct::DevBuf scan_tmp, cursor;
  hipError_t e = scan_tmp.alloc(scan_bytes);
  if (e != hipSuccess) return fail_with(sct::fail(SCT_E_NOMEM, "scan temp: %s", hipGetErrorString(e)));
  e = cursor.alloc(((size_t)1 << KEY_BITS_MAX) * 4 + 8);
  if (e != hipSuccess) return fail_with(sct::fail(SCT_E_NOMEM, "cursor: %s", hipGetErrorString(e)));
  for (int k = 0; k < p->nparts; ++k) {
    const Part pt = p->parts.p[k];
    const int64_t nkeys = 1LL << pt.key_bits;
    e = hipMalloc(&p->d_offsets[k], (size_t)(nkeys + 1) * 4);
    if (e == hipSuccess) e = hipMalloc(&p->d_bcodes[k], (size_t)std::max<int64_t>(nw, 1) * 8);
    if (e == hipSuccess) e = hipMalloc(&p->d_bindex[k], (size_t)std::max<int64_t>(nw, 1) * 4);
    if (e != hipSuccess) return fail_with(sct::fail(SCT_E_NOMEM, "bucket arrays: %s", hipGetErrorString(e)));
    uint32_t* counts = (uint32_t*)cursor.p;
    SCT_HIP(hipMemsetAsync(counts, 0, (size_t)(nkeys + 1) * 4, s));
    if (nw)
      hipLaunchKernelGGL(key_hist_kernel, dim3(grid_for(nw, 4096)), dim3(WG), 0, s, d_whitelist, nw,
                         pt, counts);
    size_t b = scan_bytes;
    e = hipcub::DeviceScan::ExclusiveSum(scan_tmp.p, b, counts, p->d_offsets[k], nkeys + 1, s);
    if (e != hipSuccess) return fail_with(sct::fail(SCT_E_HIP, "scan: %s", hipGetErrorString(e)));
    SCT_HIP(hipMemcpyAsync(counts, p->d_offsets[k], (size_t)nkeys * 4, hipMemcpyDeviceToDevice, s));
    if (nw)
      hipLaunchKernelGGL(key_scatter_kernel, dim3(grid_for(nw, 4096)), dim3(WG), 0, s, d_whitelist,
                         nw, pt, counts, p->d_bcodes[k], p->d_bindex[k]);
    SCT_LAUNCH_CHECK();
  }
  e = hipMalloc(&p->d_off_tab, sizeof(void*) * MAX_PARTS);
  if (e == hipSuccess) e = hipMalloc(&p->d_code_tab, sizeof(void*) * MAX_PARTS);
  if (e == hipSuccess) e = hipMalloc(&p->d_idx_tab, sizeof(void*) * MAX_PARTS);
  if (e != hipSuccess) return fail_with(sct::fail(SCT_E_NOMEM, "tables: %s", hipGetErrorString(e)));
  SCT_HIP(hipMemcpyAsync(p->d_off_tab, p->d_offsets, sizeof(void*) * MAX_PARTS, hipMemcpyHostToDevice, s));
  SCT_HIP(hipMemcpyAsync(p->d_code_tab, p->d_bcodes, sizeof(void*) * MAX_PARTS, hipMemcpyHostToDevice, s));
  SCT_HIP(hipMemcpyAsync(p->d_idx_tab, p->d_bindex, sizeof(void*) * MAX_PARTS, hipMemcpyHostToDevice, s));
  SCT_HIP(hipStreamSynchronize(s));  // the scratch buffers die with this call
  *out = p;
  return SCT_OK;
}

extern "C" int sct_nearest_query(sct_nearest_plan* p, const uint64_t* d_queries, int64_t nq,
                                 int32_t* d_index, uint8_t* d_dist, void* stream) {
  SCT_CHECK(p != nullptr, "plan is NULL");
  SCT_CHECK(nq >= 0, "nq must be >= 0");
  if (nq == 0) return SCT_OK;
  SCT_CHECK(d_queries && d_index && d_dist, "NULL pointer");
  hipStream_t s = sct::as_stream(stream);
  if (p->kind == 2)
    hipLaunchKernelGGL(nearest_query_kernel<2>, dim3(grid_for(nq)), dim3(WG), 0, s, d_queries, nq,
                       p->nparts, p->parts, p->d_off_tab, p->d_code_tab, p->d_idx_tab, p->max_d,
                       d_index, d_dist);
  else
    hipLaunchKernelGGL(nearest_query_kernel<3>, dim3(grid_for(nq)), dim3(WG), 0, s, d_queries, nq,
                       p->nparts, p->parts, p->d_off_tab, p->d_code_tab, p->d_idx_tab, p->max_d,
                       d_index, d_dist);
  SCT_LAUNCH_CHECK();
  return SCT_OK;
}

extern "C" int sct_nearest_host(int kind, const uint64_t* whitelist, int64_t nw, const uint64_t* queries,
                                int64_t nq, int code_bits, int max_d, int32_t* index, uint8_t* dist) {
  SCT_CHECK(nw >= 0 && nq >= 0, "bad sizes");
  sct::DevBuf dw, dq, di, dd;
  SCT_HIP(dw.alloc((size_t)nw * 8));
  if (nw) SCT_HIP(hipMemcpy(dw.p, whitelist, (size_t)nw * 8, hipMemcpyHostToDevice));
  SCT_HIP(dq.alloc((size_t)nq * 8));
  if (nq) SCT_HIP(hipMemcpy(dq.p, queries, (size_t)nq * 8, hipMemcpyHostToDevice));
  SCT_HIP(di.alloc((size_t)nq * 4));
  SCT_HIP(dd.alloc((size_t)nq));
  sct_nearest_plan* plan = nullptr;
  int rc = sct_nearest_plan_create(kind, (const uint64_t*)dw.p, nw, code_bits, max_d, nullptr, &plan);
  if (rc != SCT_OK) return rc;
  rc = sct_nearest_query(plan, (const uint64_t*)dq.p, nq, (int32_t*)di.p, (uint8_t*)dd.p, nullptr);
  sct_nearest_plan_destroy(plan);
  if (rc != SCT_OK) return rc;
  if (nq) {
    SCT_HIP(hipMemcpy(index, di.p, (size_t)nq * 4, hipMemcpyDeviceToHost));
    SCT_HIP(hipMemcpy(dist, dd.p, (size_t)nq, hipMemcpyDeviceToHost));
  }
  return SCT_OK;
}
