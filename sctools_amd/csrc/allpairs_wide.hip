// All-pairs TwoBit distance histogram for codes wider than 64 bits: the pair loop of
// Barcodes.summarize_hamming_distances (src/sctools/barcode.py:42-43) over Python ints of
// any size -- ThreeBit-encoded 22..28-bp keys (66..84 bits), TwoBit keys > 32 bp.  The
// reference's TwoBit.hamming_distance (encodings.py:113-121) counts the non-zero 2-bit
// groups of a ^ b; a 64-bit limb holds whole groups, so the distance of W-limb codes is
// the sum of popcount((x | x >> 1) & 0x5555...) over the limbs.
//
// Work items = tile pairs (a, b), a <= b, of 256-code tiles, row-major over a (contiguous
// item ranges shard across ranks like the 64-bit schemes).  A workgroup takes a contiguous
// run of items: thread t holds code 256 a + t in registers, the column tile b is staged in
// LDS (broadcast reads), and every pair adds 1 to the thread's PRIVATE LDS counter column
// hist[d][t] (bank = t mod 64: conflict-free, no atomics).  The columns are summed once per
// workgroup and added to the u64 histogram with one global atomic per bin.  W > 4 (bins >
// 129) uses one workgroup histogram with LDS atomics, flushed per item.
#include <algorithm>

#include "sct_common.h"

namespace {

constexpr int kT = 256;  // codes per tile = threads per workgroup

__device__ __forceinline__ int dist2(uint64_t x) { return __popcll((x | (x >> 1)) & 0x5555555555555555ull); }

// the even bits of x packed into 32 bits (bit 2g -> bit g)
__device__ __forceinline__ uint32_t even_bits(uint64_t x) {
  x &= 0x5555555555555555ull;
  x = (x | (x >> 1)) & 0x3333333333333333ull;
  x = (x | (x >> 2)) & 0x0F0F0F0F0F0F0F0Full;
  x = (x | (x >> 4)) & 0x00FF00FF00FF00FFull;
  x = (x | (x >> 8)) & 0x0000FFFF0000FFFFull;
  return (uint32_t)(x | (x >> 16));
}

// item t -> tile pair (a, b), items of row a: b = a .. nb-1, row a starts at a nb - a(a-1)/2
__device__ __forceinline__ void item_to_tiles(int64_t t, int64_t nb, int64_t& a, int64_t& b) {
  const double B = 2.0 * (double)nb + 1.0;
  int64_t r = (int64_t)((B - sqrt(B * B - 8.0 * (double)t)) * 0.5);
  r = r < 0 ? 0 : (r >= nb ? nb - 1 : r);
  auto start = [nb](int64_t x) { return x * nb - x * (x - 1) / 2; };
  while (r > 0 && start(r) > t) --r;
  while (r + 1 < nb && start(r + 1) <= t) ++r;
  a = r;
  b = r + (t - start(r));
}

template <int W>
__global__ __launch_bounds__(kT) void wide_private_kernel(const uint64_t* __restrict__ codes, int64_t n,
                                                          int64_t item_begin, int64_t item_end,
                                                          unsigned long long* __restrict__ hist) {
  constexpr int NB = 32 * W + 1;
  __shared__ uint32_t cnt[NB * kT];
  // the column tile as 2-bit-group planes: per code and limb {low bits, high bits} of the
  // 32 groups, so a pair's limb distance is popcount((lo ^ lo') | (hi ^ hi')): 2 ops + a
  // v_bcnt instead of the 64-bit XOR / shift / OR / AND / 2 popcounts
  __shared__ uint2 col[W * kT];
  const int t = threadIdx.x;
  for (int k = t; k < NB * kT; k += kT) cnt[k] = 0;
  const int64_t nb = (n + kT - 1) / kT;
  const int64_t span = item_end - item_begin;
  const int64_t ib = item_begin + span * blockIdx.x / gridDim.x;
  const int64_t ie = item_begin + span * (blockIdx.x + 1) / gridDim.x;
  int64_t a = 0, b = 0;
  if (ib < ie) item_to_tiles(ib, nb, a, b);
  uint32_t qlo[W], qhi[W];
  int64_t qa = -1;
  for (int64_t it = ib; it < ie; ++it) {
    if (a != qa) {  // a new row tile: this thread's code
      const int64_t i = a * kT + t;
#pragma unroll
      for (int w = 0; w < W; ++w) {
        const uint64_t x = i < n ? codes[i * W + w] : 0;
        qlo[w] = even_bits(x);
        qhi[w] = even_bits(x >> 1);
      }
      qa = a;
    }
    __syncthreads();  // the previous item's reads of col are done
    const int64_t j0 = b * kT;
    for (int k = t; k < W * kT; k += kT) {
      const int64_t j = j0 + k / W;
      const uint64_t x = j < n ? codes[j0 * W + k] : 0;
      col[k] = make_uint2(even_bits(x), even_bits(x >> 1));
    }
    __syncthreads();
    const int64_t i = a * kT + t;
    // pairs i < j: on the diagonal tile only columns above t, everywhere only j < n
    const int jfirst = a == b ? t + 1 : 0;
    const int jlast = (int)min<int64_t>(kT, n - j0);
    if (i < n) {
      for (int jj = jfirst; jj < jlast; ++jj) {
        uint32_t d = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) {
          const uint2 c = col[jj * W + w];
          d += __popc((qlo[w] ^ c.x) | (qhi[w] ^ c.y));
        }
        atomicAdd(&cnt[d * kT + t], 1u);  // private column: ds_add_u32, never contended
      }
    }
    if (++b == nb) {
      ++a;
      b = a;
    }
  }
  __syncthreads();
  for (int d = t; d < NB; d += kT) {
    unsigned long long s = 0;
    for (int k = 0; k < kT; ++k) s += cnt[d * kT + ((k + d) & (kT - 1))];
    if (s) atomicAdd(hist + d, s);
  }
}

__global__ __launch_bounds__(kT) void wide_shared_kernel(const uint64_t* __restrict__ codes, int64_t n, int W,
                                                         int64_t item_begin, int64_t item_end,
                                                         unsigned long long* __restrict__ hist) {
  extern __shared__ uint32_t smem[];  // [32 W + 1] counters, then the column tile
  const int NB = 32 * W + 1;
  uint32_t* cnt = smem;
  uint64_t* col = reinterpret_cast<uint64_t*>(smem + ((NB + 1) & ~1));
  const int t = threadIdx.x;
  for (int k = t; k < NB; k += kT) cnt[k] = 0;
  const int64_t nb = (n + kT - 1) / kT;
  const int64_t span = item_end - item_begin;
  const int64_t ib = item_begin + span * blockIdx.x / gridDim.x;
  const int64_t ie = item_begin + span * (blockIdx.x + 1) / gridDim.x;
  int64_t a = 0, b = 0;
  if (ib < ie) item_to_tiles(ib, nb, a, b);
  for (int64_t it = ib; it < ie; ++it) {
    __syncthreads();
    const int64_t j0 = b * kT;
    for (int k = t; k < W * kT; k += kT) {
      const int64_t j = j0 + k / W;
      col[k] = j < n ? codes[j0 * W + k] : 0;
    }
    __syncthreads();
    const int64_t i = a * kT + t;
    const int jfirst = a == b ? t + 1 : 0;
    const int jlast = (int)min<int64_t>(kT, n - j0);
    if (i < n) {
      for (int jj = jfirst; jj < jlast; ++jj) {
        int d = 0;
        for (int w = 0; w < W; ++w) d += dist2(codes[i * W + w] ^ col[jj * W + w]);
        atomicAdd(&cnt[d], 1u);
      }
    }
    __syncthreads();  // flush per item: at most 256 * 256 pairs in the u32 counters
    for (int d = t; d < NB; d += kT) {
      if (cnt[d]) {
        atomicAdd(hist + d, (unsigned long long)cnt[d]);
        cnt[d] = 0;
      }
    }
    if (++b == nb) {
      ++a;
      b = a;
    }
  }
}

int64_t wide_items(int64_t n) {
  const int64_t nb = (n + kT - 1) / kT;
  return nb * (nb + 1) / 2;
}

// pairs i < j inside the items [b, e) (host arithmetic over the tile pairs)
int64_t wide_range_pairs(int64_t n, int64_t b, int64_t e) {
  const int64_t nb = (n + kT - 1) / kT;
  int64_t pairs = 0, t = 0;
  for (int64_t a = 0; a < nb && t < e; ++a) {
    const int64_t ra = std::min<int64_t>(kT, n - a * kT);  // rows in tile a
    const int64_t row_items = nb - a;
    if (t + row_items <= b) {
      t += row_items;
      continue;
    }
    for (int64_t c = a; c < nb; ++c, ++t) {
      if (t < b || t >= e) continue;
      const int64_t rc = std::min<int64_t>(kT, n - c * kT);
      pairs += c == a ? ra * (ra - 1) / 2 : ra * rc;
    }
  }
  return pairs;
}

int grid_for(int64_t items) {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  return (int)std::max<int64_t>(1, std::min<int64_t>(items, (int64_t)cus * 2));
}

}  // namespace

extern "C" int sct_allpairs_wide_geometry(int64_t n, int words, int64_t* items, int* nbins) {
  SCT_CHECK(n >= 0 && words >= 1 && words <= 256, "n %lld / words %d out of range", (long long)n, words);
  if (items) *items = wide_items(n);
  if (nbins) *nbins = 32 * words + 1;
  return SCT_OK;
}

extern "C" int sct_allpairs_wide_range_pairs(int64_t n, int64_t item_begin, int64_t item_end, int64_t* pairs) {
  SCT_CHECK(pairs != nullptr && n >= 0, "bad arguments");
  SCT_CHECK(0 <= item_begin && item_begin <= item_end && item_end <= wide_items(n), "item range [%lld, %lld)",
            (long long)item_begin, (long long)item_end);
  *pairs = wide_range_pairs(n, item_begin, item_end);
  return SCT_OK;
}

extern "C" int sct_allpairs_wide(const uint64_t* d_codes, int64_t n, int words, int64_t item_begin,
                                 int64_t item_end, uint64_t* d_hist, int nbins, void* stream) {
  SCT_CHECK(words >= 1 && words <= 256, "words %d outside [1, 256]", words);
  SCT_CHECK(nbins == 32 * words + 1, "nbins must be 32 * words + 1 = %d (got %d)", 32 * words + 1, nbins);
  SCT_CHECK(n >= 0 && (n == 0 || d_codes != nullptr) && d_hist != nullptr, "NULL pointer");
  const int64_t items = wide_items(n);
  SCT_CHECK(0 <= item_begin && item_begin <= item_end && item_end <= items, "item range [%lld, %lld) of %lld",
            (long long)item_begin, (long long)item_end, (long long)items);
  if (item_begin == item_end || n < 2) return SCT_OK;
  const int grid = grid_for(item_end - item_begin);
  // private u32 counters see at most 256 pairs per item per thread
  SCT_CHECK((item_end - item_begin) / grid < (1ll << 24), "too many items per workgroup");
  hipStream_t s = sct::as_stream(stream);
  auto* h = reinterpret_cast<unsigned long long*>(d_hist);
  switch (words) {
    case 1: hipLaunchKernelGGL(wide_private_kernel<1>, dim3(grid), dim3(kT), 0, s, d_codes, n, item_begin, item_end, h); break;
    case 2: hipLaunchKernelGGL(wide_private_kernel<2>, dim3(grid), dim3(kT), 0, s, d_codes, n, item_begin, item_end, h); break;
    case 3: hipLaunchKernelGGL(wide_private_kernel<3>, dim3(grid), dim3(kT), 0, s, d_codes, n, item_begin, item_end, h); break;
    case 4: hipLaunchKernelGGL(wide_private_kernel<4>, dim3(grid), dim3(kT), 0, s, d_codes, n, item_begin, item_end, h); break;
    default: {
      const size_t shm = (size_t)((nbins + 1) & ~1) * 4 + (size_t)words * kT * 8;
      SCT_CHECK(shm <= 160 * 1024, "codes of %d limbs need %zu B of LDS", words, shm);
      if (shm > 64 * 1024)
        SCT_HIP(hipFuncSetAttribute((const void*)wide_shared_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)shm));
      hipLaunchKernelGGL(wide_shared_kernel, dim3(grid), dim3(kT), shm, s, d_codes, n, words, item_begin, item_end, h);
    }
  }
  SCT_LAUNCH_CHECK();
  return SCT_OK;
}

extern "C" int sct_hamming_hist_allpairs_wide_host(const uint64_t* codes, int64_t n, int words, uint64_t* hist,
                                                   int nbins) {
  SCT_CHECK(hist != nullptr && (n == 0 || codes != nullptr), "NULL pointer");
  SCT_CHECK(words >= 1 && words <= 256 && nbins == 32 * words + 1, "words %d / nbins %d", words, nbins);
  for (int d = 0; d < nbins; ++d) hist[d] = 0;
  if (n < 2) return SCT_OK;
  sct::DevBuf dc, dh;
  SCT_HIP(dc.alloc((size_t)n * words * 8));
  SCT_HIP(dh.alloc((size_t)nbins * 8));
  SCT_HIP(hipMemcpy(dc.p, codes, (size_t)n * words * 8, hipMemcpyHostToDevice));
  SCT_HIP(hipMemset(dh.p, 0, (size_t)nbins * 8));
  const int rc = sct_allpairs_wide((const uint64_t*)dc.p, n, words, 0, wide_items(n), (uint64_t*)dh.p, nbins, nullptr);
  if (rc != SCT_OK) return rc;
  SCT_HIP(hipMemcpy(hist, dh.p, (size_t)nbins * 8, hipMemcpyDeviceToHost));
  return SCT_OK;
}
