// Bench aid: the streaming HBM copy the library's kernels are priced against beside the
// 8 TB/s spec (bench.py `copy_ceiling_gbs`).  One 16-B element per lane and one pass over the
// data (a workgroup per 4 KiB): the form that reaches the guide's ~6.3 TB/s float4 copy
// (MI355X_MICROARCH.md).  A resident grid looping over the data with 1-8 loads in flight per
// lane stays at 4.7-5.0 TB/s, plain or nontemporal (tools/copy_probe.hip,
// profiles/copy_probe_r04.json): the round-3 form of this kernel, whose 4.8 TB/s overstated
// every frac_of_copy_ceiling by ~30 %.
#include <algorithm>

#include "sct_common.h"

namespace {

typedef unsigned v4u __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void stream_copy_kernel(const v4u* __restrict__ src, v4u* __restrict__ dst,
                                                          int64_t n16) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n16) dst[i] = src[i];
}

}  // namespace

extern "C" int sct_stream_copy(void* dst, const void* src, int64_t bytes, void* stream) {
  SCT_CHECK(bytes >= 0 && bytes % 16 == 0, "bytes must be a multiple of 16");
  SCT_CHECK(bytes == 0 || (dst && src), "NULL pointer");
  if (bytes == 0) return SCT_OK;
  const int64_t n16 = bytes / 16;
  SCT_CHECK(sct::ceil_div(n16, 256) < (1LL << 31), "copy too large for one launch");
  hipLaunchKernelGGL(stream_copy_kernel, dim3((unsigned)sct::ceil_div(n16, 256)), dim3(256), 0, sct::as_stream(stream),
                     reinterpret_cast<const v4u*>(src), reinterpret_cast<v4u*>(dst), n16);
  SCT_LAUNCH_CHECK();
  return SCT_OK;
}
