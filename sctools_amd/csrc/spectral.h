// SCT_ALLPAIRS_SPECTRAL: internal interface between the plan (allpairs.hip) and the
// Walsh-Hadamard kernels (spectral.hip).  DESIGN.md §3.8.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sct_spectral {

constexpr int kSpaceBits = 32;                 // 16 bases: codes are points of Z_2^32
constexpr int kLoBits = 20;                    // element index inside a slice
constexpr int kSlices = 1 << (kSpaceBits - kLoBits);  // work items: z >> 20
constexpr int kNCounts = 1 + 17;               // [n, S_0..S_16]

// Device state of a SPECTRAL plan (owned by sct_allpairs_plan).
struct State {
  int64_t n = 0;
  uint64_t* d_sorted = nullptr;  // codes sorted by their low 20 bits
  uint16_t* d_hi = nullptr;      // code >> 20, in that order
  uint32_t* d_off = nullptr;     // [2^20 + 1] first code of each low-20-bit value
  int32_t* d_buf = nullptr;      // chunk slices x 2^20 transform values
  int64_t chunk = 0;             // slices per pass
  void* d_sort_tmp = nullptr;
  size_t sort_tmp_bytes = 0;
  int grid = 0;                  // persistent grid of the square/reduce pass
};

// allocate (chunk = slices held in HBM at once); returns an SCT_* code
int create(State& st, int64_t n, int64_t chunk, int cus);
void destroy(State& st);
// sort + split the codes (any slice range needs all of them)
int build(State& st, const uint64_t* d_codes, hipStream_t s);
// add the counts of slices [z_begin, z_end): d_counts[1 + w] += S_w over those slices,
// d_counts[0] += n when z_begin == 0
int count(State& st, int64_t z_begin, int64_t z_end, unsigned long long* d_counts, hipStream_t s);

}  // namespace sct_spectral
