// SCT_ALLPAIRS_SPECTRAL: internal interface between the plan (allpairs.hip) and the
// Walsh-Hadamard kernels (spectral.hip).  DESIGN.md §3.8.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

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
  bool mfma = true;              // int8 seeds: first 6 butterfly levels on the matrix cores
  uint16_t* d_order = nullptr;   // [2^17]: at [L, 2L) the offsets [0, L) sorted by digit weight
  int tile_wgs = 2;              // resident MFMA-tile workgroups per CU
  int tile_reg = 0;              // int8 seeds: the register-resident tile (one wave per slice), variant
  int tile_reg_wgs = 2;          // its resident workgroups per CU
  bool seed_db = false;          // int8 walk seed: double-buffered byte stage
  bool seed_spread = false;      // int8 seeds: stores spread over the walk (16-slice blocks)
  void* d_mx = nullptr;          // int8 seeds: the MFMA seed's operand tables (null: the walk seed)
  int mx_form = 2;               // the MFMA seed's workgroup shape (A/B)
  int ilv = 0;                   // int8: the direct MFMA seed + G-slice interleaved intermediate (G)
  // seed / tile overlap: chunk j+1's seed (side stream, second buffer) runs beside chunk j's tile
  bool overlap = false;
  void* d_buf2 = nullptr;
  hipStream_t side = nullptr;
  hipEvent_t ev[5] = {};         // [0, 1] tile done with buffer 0 / 1, [2, 3] seed done, [4] start
  void* d_buf = nullptr;         // chunk slices x 2^14 seed values
  int64_t chunk = 0;             // slices per pass
  int grid = 0;                  // compute units (the tile kernel's persistent grid)
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
