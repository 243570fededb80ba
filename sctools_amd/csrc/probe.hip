// Bench aid: the streaming HBM copy the library's kernels are priced against beside the
// 8 TB/s spec (bench.py `copy_ceiling_gbs`).  A resident grid of 256-thread workgroups copies
// 16 B per lane per load, four loads in flight per lane, nontemporal both ways, so the
// figure is what a plain read + write stream reaches on this device (MI355X_MICROARCH.md:
// about 6.3 TB/s), not a torch / runtime blit.
#include <algorithm>

#include "sct_common.h"

namespace {

typedef unsigned v4u __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void stream_copy_kernel(const v4u* __restrict__ src, v4u* __restrict__ dst,
                                                          int64_t n16) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    v4u v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = __builtin_nontemporal_load(src + i + k * stride);
#pragma unroll
    for (int k = 0; k < 4; ++k) __builtin_nontemporal_store(v[k], dst + i + k * stride);
  }
  for (; i < n16; i += stride) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

}  // namespace

extern "C" int sct_stream_copy(void* dst, const void* src, int64_t bytes, void* stream) {
  SCT_CHECK(bytes >= 0 && bytes % 16 == 0, "bytes must be a multiple of 16");
  SCT_CHECK(bytes == 0 || (dst && src), "NULL pointer");
  if (bytes == 0) return SCT_OK;
  int dev = 0, cus = 256;
  SCT_HIP(hipGetDevice(&dev));
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  const int64_t n16 = bytes / 16;
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((int64_t)cus * 8, sct::ceil_div(n16, 256)));
  hipLaunchKernelGGL(stream_copy_kernel, dim3(grid), dim3(256), 0, sct::as_stream(stream),
                     reinterpret_cast<const v4u*>(src), reinterpret_cast<v4u*>(dst), n16);
  SCT_LAUNCH_CHECK();
  return SCT_OK;
}
