// Internal helpers shared by the libsctools_hip.so translation units.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdarg.h>
#include <stdio.h>

#include <functional>
#include <vector>

#include "../../include/sctools_hip.h"

namespace sct {

// Thread-local last-error buffer behind sct_last_error().
void set_error(const char* fmt, ...);
const char* last_error();

inline int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  set_error("%s", buf);
  return code;
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// RAII device buffer for the *_host convenience entry points.
struct DevBuf {
  void* p = nullptr;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  hipError_t alloc(size_t bytes) { return hipMalloc(&p, bytes ? bytes : 1); }
};

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Per-thread, per-device staging of the *_host entry points (host.cpp): one non-blocking
// stream, one page-locked host-coherent buffer and one device buffer, created on first use
// and grown on demand (never freed: process exit reclaims them), so a drop-in scalar call
// costs a launch and a stream sync instead of hipMalloc / hipFree per argument.
struct HostStage {
  int device = -1;
  hipStream_t stream = nullptr;
  uint8_t* pinned = nullptr;  // hipHostMallocCoherent: kernels may read / write it directly
  uint8_t* pinned_dev = nullptr;  // the same buffer as the device sees it
  size_t pinned_cap = 0;
  uint8_t* dev = nullptr;
  size_t dev_cap = 0;
  // the host stream paths' pipeline streams (sct_encode_stream_host), created on first use and
  // kept: a stream's creation and destruction cost more than a piece's copies (round 5)
  hipStream_t pipe[3] = {nullptr, nullptr, nullptr};
};
// nullptr (with the error set) if the stage cannot be created.
HostStage* host_stage();
// True when all of [p, p + bytes) lies in ONE page-locked host allocation the HIP runtime knows
// (hipHostMalloc, torch pin_memory, a caller's own hipHostRegister): DMA may then use the caller's
// memory directly.  The library itself never registers or unregisters caller memory -- pageable
// arrays are copied through the stage's own pinned buffer instead.
bool host_range_pinned(const void* p, size_t bytes);
int stage_reserve(HostStage* st, size_t pinned_bytes, size_t dev_bytes);
// memcpy split over the library's copy helper threads for large pageable <-> page-locked copies
// (host.cpp); small copies, or one while another thread's is running, stay on the calling thread
void par_memcpy(void* dst, const void* src, size_t bytes);
// the calling thread's stage on the current device gives its device buffer back (the next call
// that needs one maps it again)
void stage_release_device();
// Calls of at most this many bytes (inputs + outputs) run zero-copy on the pinned buffer.
constexpr size_t kZeroCopyBytes = 64 << 10;
// Larger calls up to this size go through the pinned + device buffers (two copies); beyond
// it the caller's arrays are copied through per-call device allocations.
constexpr size_t kStageBytes = 256ull << 20;

// Stream-ordered scratch from the library's private memory pool of the current device (host.cpp;
// the device's default pool is not touched): released memory stays in the pool for the next call.
hipError_t pool_alloc(void** p, size_t bytes, hipStream_t s);
// every pool's idle memory back to the device (sct_allpairs_cache_release)
void pool_trim();
void pool_free(void* p, hipStream_t s);

// Several devices from one process (devices.cpp): fn(r) for every slot r in [0, ndev) on a
// persistent worker thread of its own (slot r is always the same thread, so its thread-local host
// stages and pipeline streams are reused from call to call) with devices[r] its current device;
// devices == NULL or ndev <= 1 runs fn(0) on the calling thread and its current device.
// Returns the first failing slot's status with its message.  One such call at a time per process.
int run_on_devices(const int* devices, int ndev, const std::function<int(int)>& fn);

// sct_tune_set value of `key`, or dflt when unset (host.cpp).
int64_t tune(int key, int64_t dflt);

// Stop the resident scalar servers (encode.hip) before a launch whose grid is sized to the
// resident workgroups, so none of its workgroups waits behind a server wave's registers.
// Cheap when no server runs.
void scalar_quiesce();

// Bench aid: per-launch HIP-event timing of a plan's kernels on the stream each launch runs on
// (sct_allpairs_timing).  Off by default; when on, start() records an event before a launch
// and stop() one after it, and collect() waits for the recorded pairs and sums their spans
// per kind.  Events are pooled, so a timed run allocates nothing after its first steps.
struct LaunchTimer {
  enum Kind { SEED = 0, TILE = 1, COUNT = 2, BUILD = 3, NKINDS = 4 };
  bool on = false;
  double ms[NKINDS] = {};
  int64_t launches[NKINDS] = {};
  struct Rec {
    hipEvent_t a, b;
    int kind;
  };
  std::vector<Rec> pending;
  std::vector<hipEvent_t> pool;

  hipEvent_t take() {
    hipEvent_t e = nullptr;
    if (!pool.empty()) {
      e = pool.back();
      pool.pop_back();
    } else if (hipEventCreate(&e) != hipSuccess) {
      e = nullptr;
    }
    return e;
  }
  hipEvent_t start(hipStream_t s) {
    if (!on) return nullptr;
    hipEvent_t a = take();
    if (a) (void)hipEventRecord(a, s);
    return a;
  }
  void stop(hipStream_t s, hipEvent_t a, int kind) {
    if (!on || !a) return;
    hipEvent_t b = take();
    if (!b) return;
    (void)hipEventRecord(b, s);
    pending.push_back(Rec{a, b, kind});
  }
  void collect() {
    for (const Rec& r : pending) {
      float t = 0;
      if (hipEventSynchronize(r.b) == hipSuccess && hipEventElapsedTime(&t, r.a, r.b) == hipSuccess) {
        ms[r.kind] += t;
        launches[r.kind] += 1;
      }
      pool.push_back(r.a);
      pool.push_back(r.b);
    }
    pending.clear();
  }
  void reset() {
    collect();
    for (auto& v : ms) v = 0;
    for (auto& v : launches) v = 0;
  }
  ~LaunchTimer() {
    for (const Rec& r : pending) {
      (void)hipEventDestroy(r.a);
      (void)hipEventDestroy(r.b);
    }
    for (hipEvent_t e : pool) (void)hipEventDestroy(e);
  }
};

// Moment-assisted all-pairs scheme (SCT_ALLPAIRS_MOMENTS, 16-base TwoBit codes):
// the count kernel accumulates only these 13 subset products of the distance bits
// d0..d3 (d mod 16), and the agreement moments M_k = sum over pairs of C(16 - d, k),
// k = 1..kMomOrder, are counted from the codes' 1/2/3-position marginals.  With the
// pair count, that is 1 + 13 + 3 = 17 independent linear functionals of hist[0..16]
// (the product set is a minimum one for moments of order <= 3).
constexpr int kMomG = 16;  // base positions (distance 0..16)
constexpr int kMomOrder = 3;
constexpr int kMomNProd = 13;
constexpr int kMomProducts[kMomNProd] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15};
constexpr int kMomNCounts = 1 + kMomNProd + kMomOrder;  // [pairs, products..., M1, M2, M3]

}  // namespace sct

#define SCT_HIP(call)                                                                        \
  do {                                                                                       \
    hipError_t e_ = (call);                                                                  \
    if (e_ != hipSuccess)                                                                    \
      return ::sct::fail(e_ == hipErrorOutOfMemory ? SCT_E_NOMEM : SCT_E_HIP, "%s: %s (%s:%d)", \
                         #call, hipGetErrorString(e_), __FILE__, __LINE__);                  \
  } while (0)

#define SCT_CHECK(cond, ...)                                 \
  do {                                                       \
    if (!(cond)) return ::sct::fail(SCT_E_INVALID, __VA_ARGS__); \
  } while (0)

#define SCT_LAUNCH_CHECK()                                                                      \
  do {                                                                                          \
    hipError_t e_ = hipGetLastError();                                                          \
    if (e_ != hipSuccess)                                                                       \
      return ::sct::fail(SCT_E_HIP, "kernel launch: %s (%s:%d)", hipGetErrorString(e_), __FILE__, \
                         __LINE__);                                                             \
  } while (0)
