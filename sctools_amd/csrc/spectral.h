// SCT_ALLPAIRS_SPECTRAL: internal interface between the plan (allpairs.hip) and the
// Walsh-Hadamard kernels (spectral.hip).  DESIGN.md §3.8.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>
#include <vector>

#include "sct_common.h"

namespace sct_spectral {

constexpr int kSpaceBits = 32;                 // 16 bases: codes are points of Z_2^32
constexpr int kLoBits = 14;                    // element index inside a slice (one LDS tile)
constexpr int kSlices = 1 << (kSpaceBits - kLoBits);  // work items: z >> 14
// SPECTRAL counts: [n, sum f^2, then S_w (w = 0..16) as three limbs summed separately]:
//   counts[kLimb0 + w] += bits 0..31, counts[kLimb1 + w] += bits 32..63 and
//   counts[kLimb2 + w] += bits 64.. of every partial sum a workgroup adds, so no limb
//   ever carries (each add is < 2^32 or small) and S_w = l0 + 2^32 l1 + 2^64 l2 stays exact
//   for any multiset (sum_w S_w = 2^32 sum f^2 can exceed 2^64), also after an int64
//   all-reduce of the counts over ranks.  sum f^2 (the ordered pairs of equal codes, self
//   pairs included) is computed independently from the sorted codes, so the host checks
//   sum_w S_w == 2^32 sum f^2 exactly.
constexpr int kNCounts = 2 + 3 * 17;
constexpr int kLimb0 = 2, kLimb1 = kLimb0 + 17, kLimb2 = kLimb1 + 17;

// counts[limbs of S_w] += lo + 2^32 hi (lo, hi: LDS partial sums of 32-bit pieces, or a 64-bit
// value split as lo = v & 0xFFFFFFFF, hi = v >> 32; lo < 2^63, hi < 2^63)
__device__ __forceinline__ void add_weight_sum(unsigned long long* counts, int w, unsigned long long lo,
                                               unsigned long long hi) {
  const unsigned long long b = hi + (lo >> 32);
  if (lo & 0xFFFFFFFFull) atomicAdd(counts + kLimb0 + w, lo & 0xFFFFFFFFull);
  if (b & 0xFFFFFFFFull) atomicAdd(counts + kLimb1 + w, b & 0xFFFFFFFFull);
  if (b >> 32) atomicAdd(counts + kLimb2 + w, b >> 32);
}
__device__ __forceinline__ void add_weight_sum64(unsigned long long* counts, int w, unsigned long long v) {
  add_weight_sum(counts, w, v & 0xFFFFFFFFull, v >> 32);
}
// the job's constants, once (by the launch holding slice 0): n and sum f^2
__device__ __forceinline__ void add_job_constants(unsigned long long* counts, unsigned long long add_n,
                                                  const unsigned long long* sumsq) {
  if (add_n && blockIdx.x == 0 && threadIdx.x == 0) {
    atomicAdd(counts, add_n);
    atomicAdd(counts + 1, sumsq ? *sumsq : add_n);  // no sumsq: the caller promised distinct codes
  }
}

// non-zero 2-bit digits of z
__device__ __forceinline__ int digit_weight(uint32_t z) {
  return __popc((z | (z >> 1)) & 0x55555555u);
}
constexpr int digit_weight_c(uint32_t z) {
  int w = 0;
  for (; z; z >>= 2) w += (z & 3) != 0;
  return w;
}
constexpr int gray(int i) { return i ^ (i >> 1); }
// a + popcount(x) as one v_bcnt_u32_b32 with the running sum as its addend: the compiler
// otherwise counts every group from 0 and sums the counts with v_add3 (one more VALU
// instruction per walk step)
__device__ __forceinline__ uint32_t popc_add(uint32_t x, uint32_t a) {
  uint32_t r;
  asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(a));
  return r;
}

// The column (offset in the block of 256) lane `tid` walks: the block's columns in three classes by
// group count -- >= 3, 2, <= 1 -- each class in column order (a stable partition: ballots within a
// wave, counts across the 4 waves), so the columns of more than 64 codes share waves instead of
// raising every wave's walk to 3 groups, and the stage bytes a 32-lane group stores stay mostly
// increasing (2-way bank conflicts at most, free for a byte store).  Each column's result still goes
// to its own stage byte: only which lane walks which column changes.  Two barriers.
__device__ __forceinline__ int seed_lane_column(const uint32_t* __restrict__ gofs, int c0, int tid) {
  __shared__ uint32_t s_wcnt[4][3];
  __shared__ uint8_t s_col[256];
  const uint32_t ng = gofs[c0 + tid + 1] - gofs[c0 + tid];
  const int cls = ng >= 3u ? 0 : (ng == 2u ? 1 : 2);
  const int lane = tid & 63, wave = tid >> 6;
  const uint64_t b0 = __ballot(cls == 0), b1 = __ballot(cls == 1), b2 = __ballot(cls == 2);
  const uint64_t mine = cls == 0 ? b0 : (cls == 1 ? b1 : b2);
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;  // the lanes before this one
  if (lane == 0) {
    s_wcnt[wave][0] = (uint32_t)__popcll(b0);
    s_wcnt[wave][1] = (uint32_t)__popcll(b1);
    s_wcnt[wave][2] = (uint32_t)__popcll(b2);
  }
  __syncthreads();
  uint32_t pos = (uint32_t)__popcll(mine & below);
  for (int k = 0; k < cls; ++k)
    for (int w = 0; w < 4; ++w) pos += s_wcnt[w][k];
  for (int w = 0; w < wave; ++w) pos += s_wcnt[w][cls];
  s_col[pos] = (uint8_t)tid;
  __syncthreads();
  return (int)s_col[tid];
}
constexpr int ctz_c(int i) {
  int k = 0;
  while (!(i & 1)) {
    i >>= 1;
    ++k;
  }
  return k;
}

// Per-device cache of an all-pairs plan's device buffers (DESIGN.md §3.8 "plan cache"): a plan
// created while its device's workspace is idle borrows it -- its buffers are grow-only slots kept
// across plans, so a one-shot call (plan create, build, count, destroy) maps no memory after the
// first one: no 4 GiB hipMalloc / hipFree, no order-table upload.  A plan created while the
// workspace is lent out (a second live plan on the device) allocates its own buffers as before.
// sct_allpairs_cache_release() frees the idle workspaces.
enum WsSlot {
  W_CODES, W_HI, W_OFF, W_CNT, W_GOFS, W_HIST, W_PLANES, W_BUF, W_SUMSQ, W_SUMSQ_TMP, W_PROBE, W_ORDER,
  W_COUNTS, W_NSLOTS
};
struct Workspace;
// the current device's workspace, lent to the caller, or nullptr when it is lent out already
Workspace* ws_acquire();
// give it back (its buffers stay allocated unless a release was asked for meanwhile; a private
// arena is freed)
void ws_release(Workspace* ws);
// a private arena of one `bytes` block for one plan (never shared; freed by ws_release)
Workspace* ws_arena(size_t bytes);
// slot `slot` of at least `bytes` (grow-only); ws == nullptr: a plain hipMalloc
int ws_get(Workspace* ws, int slot, size_t bytes, void** p);
// free p unless it came from a workspace
void ws_put(Workspace* ws, void* p);
// the digit-weight order table is the same for every plan: uploaded once per workspace
bool* ws_order_ready(Workspace* ws);
// free every idle workspace (all devices); one lent out is freed when its plan returns it
void ws_release_all();

// Device state of a SPECTRAL plan (owned by sct_allpairs_plan).
struct State {
  Workspace* ws = nullptr;       // the borrowed workspace, or nullptr (buffers owned)
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
  size_t buf_bytes = 0;
  int64_t chunk = 0;             // slices per pass
  int grid = 0;                  // compute units (the tile kernel's persistent grid)
  sct::LaunchTimer* timer = nullptr;  // the plan's (bench aid), not owned
  // 16-bit columns (spectral16.hip): sets whose densest 14-bit column needs int16 seeds but
  // whose densest 16-bit column holds <= 127 codes run the transform as 2^16 slices x 2^16
  // columns with int8 seeds; the plan's items stay 2^18 virtual slices (4 per real slice)
  int lo_bits = 14;
  int64_t chunk16 = 0;           // real 16-bit slices per pass
  // sum f^2 of the plan's codes (device word), computed by the plan's first build
  unsigned long long* d_sumsq = nullptr;
  bool sumsq_ready = false;
  // the caller promised pairwise-distinct codes (SCT_ALLPAIRS_DISTINCT): sum f^2 = n, no sort;
  // a broken promise fails the host's exact check sum_w S_w == 2^32 n, never a silent result
  bool distinct = false;
  const unsigned long long* sumsq_ptr() const { return distinct ? nullptr : d_sumsq; }
  void* d_sumsq_tmp = nullptr;   // sort scratch when the intermediate is too small to lend it
  // streams the plan enqueued work on, each with an event recorded after its last enqueue: a
  // borrowed workspace goes back only once they have passed (the next plan may use another stream)
  std::vector<std::pair<hipStream_t, hipEvent_t>> used;
};
// record that work of the plan was enqueued on s (call after the enqueue)
void note_stream(State& st, hipStream_t s);

// d_sumsq = sum over distinct codes of multiplicity^2 (radix sort of the low 32 bits + a
// lower-bound pass), once per plan, on stream s (the intermediate d_buf is the scratch)
int ensure_sumsq(State& st, const uint64_t* d_codes, hipStream_t s);

constexpr int kLoBits16 = 16;
constexpr int kSlices16 = 1 << (kSpaceBits - kLoBits16);

// the 16-bit column path (spectral16.hip); the functions below dispatch to it when
// st.lo_bits == 16.  max16: codes in the densest 16-bit column (<= 127); chunk in virtual
// slices (4 per real one).
int create16(State& st, const uint64_t* d_codes, int64_t n, unsigned max16, int64_t chunk, int cus);
// the intermediate of `bytes`, halved (with *chunk) while the device cannot hold it, down to a
// floor of `min_chunk` slices (a smaller chunk only costs launches)
int alloc_buf(State& st, int64_t* chunk, int64_t min_chunk, size_t bytes_per_slice);
int build16(State& st, const uint64_t* d_codes, hipStream_t s);
int count16(State& st, int64_t z_begin, int64_t z_end, unsigned long long* d_counts, hipStream_t s);
int time_kernels16(State& st, int64_t z_begin, int64_t z_end, unsigned long long* d_counts, int repeats,
                   hipStream_t s, double* seed_ms, double* tile_ms, int64_t* slices);
// codes in the densest column of the low `lo_bits` bits (device scratch of 2^lo_bits words)
int max_column(const uint64_t* d_codes, int64_t n, int lo_bits, unsigned* out);
// the digit-weight slice order tables (st.d_order)
int make_order_table(State& st);

// allocate (chunk = slices held in HBM at once) and size the intermediate from the
// codes' densest column (max14 / max16: codes in the densest 14- / 16-bit column, from the
// plan's probe); returns an SCT_* code
int create(State& st, const uint64_t* d_codes, int64_t n, int64_t chunk, int cus, unsigned max14, unsigned max16);
// one pass over the codes: their OR and the densest 14- and 16-bit columns, into out[0..2]
// (host; one synchronisation); scratch from the plan's workspace slot W_PROBE
int probe(Workspace* ws, const uint64_t* d_codes, int64_t n, unsigned long long* out);
void destroy(State& st);
// wait for every piece of work the plan enqueued (its recorded streams' events)
void wait_idle(State& st);
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
