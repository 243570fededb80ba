// SCT_ALLPAIRS_SPECTRAL: internal interface between the plan (allpairs.hip) and the
// Walsh-Hadamard kernels (spectral.hip).  DESIGN.md §3.8.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sct_common.h"

namespace sct_spectral {

constexpr int kSpaceBits = 32;                 // 16 bases: codes are points of Z_2^32
constexpr int kLoBits = 14;                    // element index inside a slice (one LDS tile)
constexpr int kSlices = 1 << (kSpaceBits - kLoBits);  // work items: z >> 14
constexpr int kNCounts = 1 + 17;               // [n, S_0..S_16]

// Device state of a SPECTRAL plan (owned by sct_allpairs_plan).
struct State {
  int64_t n = 0;
  uint32_t* d_hi = nullptr;      // code >> 14 of every code, grouped by column (low 14 bits)
  uint32_t* d_off = nullptr;     // [2^14 + 1] first code of each low-14-bit column
  uint32_t* d_cnt = nullptr;     // [2][2^14] column counts
  uint32_t* d_hist = nullptr;    // [128][2^14] per-workgroup column counts -> prefixes (build)
  unsigned max_m = 0;            // codes in the densest column
  uint32_t* d_gofs = nullptr;    // [2^14 + 1] first 32-code group of each column
  uint32_t* d_planes = nullptr;  // [groups][18] bit planes of the groups' code >> 14
  int64_t max_groups = 0;
  int elem_bytes = 1;            // seed -> tile intermediate: int8 / int16 / int32
  uint16_t* d_order = nullptr;   // [2^17]: at [L, 2L) the offsets [0, L) sorted by digit weight
  int tile_wgs = 2;              // resident register-tile workgroups per CU
  void* d_buf = nullptr;         // chunk slices x 2^14 seed values
  int64_t chunk = 0;             // slices per pass
  int grid = 0;                  // compute units (the tile kernel's persistent grid)
  sct::LaunchTimer* timer = nullptr;  // the plan's (bench aid), not owned
};

// allocate (chunk = slices held in HBM at once) and size the intermediate from the
// codes' densest column; returns an SCT_* code
int create(State& st, const uint64_t* d_codes, int64_t n, int64_t chunk, int cus);
void destroy(State& st);
// group the codes by column + bit planes (any slice range needs all of them)
int build(State& st, const uint64_t* d_codes, hipStream_t s);
// add the counts of slices [z_begin, z_end): d_counts[1 + w] += S_w over those slices,
// d_counts[0] += n when z_begin == 0
int count(State& st, int64_t z_begin, int64_t z_end, unsigned long long* d_counts, hipStream_t s);

// bench aid: ms per launch of the seed and tile kernels over the first chunk of
// [z_begin, z_end) (`slices` of them), each timed as `repeats` back-to-back launches
int time_kernels(State& st, int64_t z_begin, int64_t z_end, unsigned long long* d_counts, int repeats,
                 hipStream_t s, double* seed_ms, double* tile_ms, int64_t* slices);

}  // namespace sct_spectral
