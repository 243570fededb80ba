// Where does a scalar drop-in call's time go?  Ping-pong floors of the mailbox
// shapes the scalar server could use, against the library's own C call in a tight loop:
//   dword      one lane polls one dword, answers one dword (tools/vram_host_probe.hip's floor)
//   line       16 lanes poll the 64-B request line, one lane answers one dword
//   line_resp  16 lanes poll the line, 16 lanes answer a 64-B line
//   line2      as line_resp with the next poll issued before this one is examined
//   split2/4   2 / 4 polls in flight, each on its own copy of the request line (256 B apart; the
//              host writes every copy)
//   c_call     sct_hamming_pairs_host(kind 2, one pair) through the library named by $SCTOOLS_HIP_LIB
//              (default sctools_amd/libsctools_hip.so)
//   get_device hipGetDevice alone
//   hipcc --offload-arch=gfx950 -O2 tools/scalar_floor_probe.hip -o tools/scalar_floor_probe -ldl \
//     && tools/scalar_floor_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <chrono>
#include <vector>

typedef int (*hamming_fn)(int, const uint64_t*, const uint64_t*, int64_t, int, int32_t*);
typedef int (*stop_fn)(void);
typedef int (*decode2_fn)(const uint64_t*, int64_t, int, int, uint8_t*);
typedef int (*gc_fn)(int, const uint64_t*, int64_t, int, int, int32_t*);

#define CHK(x)                                               \
  do {                                                       \
    hipError_t e = (x);                                      \
    if (e != hipSuccess) {                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); \
      return 1;                                              \
    }                                                        \
  } while (0)

__device__ __forceinline__ uint32_t sys_load(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void sys_store(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// mode 0 dword, 1 line, 2 line_resp, 3 line2; req[0] = seq, answered in resp[0]; exits after
// `rounds` answers or ~2^26 idle polls
__global__ __launch_bounds__(64) void ping(uint32_t* req, uint32_t* resp, int rounds, int mode) {
  const int lane = threadIdx.x;
  uint32_t last = 0;
  const int width = mode == 0 ? 1 : 16;
  uint32_t line = lane < width ? sys_load(&req[lane]) : 0u;
  for (int r = 0; r < rounds;) {
    uint64_t spins = 0;
    uint32_t seq;
    for (;;) {
      uint32_t ahead = 0;
      if (mode == 3 && lane < width) ahead = sys_load(&req[lane]);
      seq = __builtin_amdgcn_readlane(line, 0);
      if (seq != last) {
        if (mode == 3) line = ahead;
        break;
      }
      if (++spins > (1ull << 26)) return;
      line = mode == 3 ? ahead : (lane < width ? sys_load(&req[lane]) : 0u);
    }
    last = seq;
    ++r;
    if (mode == 2 || mode == 3) {
      if (lane < 16) sys_store(&resp[lane], lane == 0 ? seq : __builtin_amdgcn_readlane(line, lane & 15));
    } else if (lane == 0) {
      sys_store(&resp[0], seq);
    }
    if (mode != 3) line = lane < width ? sys_load(&req[lane]) : 0u;
  }
}

// K polls in flight, poll j on copy j % K of the line (copies 64 dwords apart)
template <int K>
__global__ __launch_bounds__(64) void ping_split(uint32_t* req, uint32_t* resp, int rounds) {
  const int lane = threadIdx.x;
  uint32_t last = 0;
  uint32_t v[K];
#pragma unroll
  for (int j = 0; j < K; ++j) v[j] = sys_load(&req[64 * j + (lane & 15)]);  // no lane branch: exact waits
  uint64_t spins = 0;
  for (int r = 0; r < rounds;) {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const uint32_t seq = __builtin_amdgcn_readlane(v[j], 0);
      const uint32_t mine = v[j];
      v[j] = sys_load(&req[64 * j + (lane & 15)]);
      if (seq != last && seq > last) {
        last = seq;
        ++r;
        if (lane < 16) sys_store(&resp[lane], lane == 0 ? seq : __builtin_amdgcn_readlane(mine, lane & 15));
        spins = 0;
      }
    }
    if (++spins > (1ull << 26)) return;
  }
}

static double pingpong(uint32_t* req_h, uint32_t* req_d, uint32_t* resp_h, uint32_t* resp_d, int rounds, int mode,
                       hipStream_t s) {
  __atomic_store_n(&req_h[0], 0u, __ATOMIC_RELEASE);
  __atomic_store_n(&resp_h[0], 0u, __ATOMIC_RELEASE);
  const int copies = mode == 4 ? 2 : mode == 5 ? 4 : 1;
  for (int j = 0; j < copies; ++j) __atomic_store_n(&req_h[64 * j], 0u, __ATOMIC_RELEASE);
  if (mode == 4)
    hipLaunchKernelGGL(ping_split<2>, dim3(1), dim3(64), 0, s, req_d, resp_d, rounds);
  else if (mode == 5)
    hipLaunchKernelGGL(ping_split<4>, dim3(1), dim3(64), 0, s, req_d, resp_d, rounds);
  else
    hipLaunchKernelGGL(ping, dim3(1), dim3(64), 0, s, req_d, resp_d, rounds, mode);
  std::vector<double> per;
  per.reserve(rounds);
  for (uint32_t r = 1; r <= (uint32_t)rounds; ++r) {
    const auto t0 = std::chrono::steady_clock::now();
    for (int j = 0; j < copies; ++j) {
      for (int k = 1; k < 15; ++k) req_h[64 * j + k] = r * 16 + k;  // the fields a real request writes
      __atomic_store_n(&req_h[64 * j], r, __ATOMIC_RELEASE);
    }
    uint64_t spins = 0;
    while (__atomic_load_n(&resp_h[0], __ATOMIC_ACQUIRE) != r)
      if (++spins > (1ull << 32)) return -1.0;
    per.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  }
  (void)hipStreamSynchronize(s);
  std::sort(per.begin(), per.end());
  return per[per.size() / 2];
}

int main() {
  CHK(hipSetDevice(0));
  hipStream_t s;
  CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  uint32_t *req_h, *req_d, *resp_h, *resp_d;
  CHK(hipHostMalloc((void**)&req_h, 4096, hipHostMallocCoherent | hipHostMallocMapped));
  CHK(hipHostGetDevicePointer((void**)&req_d, req_h, 0));
  CHK(hipHostMalloc((void**)&resp_h, 4096, hipHostMallocCoherent | hipHostMallocMapped));
  CHK(hipHostGetDevicePointer((void**)&resp_d, resp_h, 0));
  const char* names[] = {"dword", "line", "line_resp", "line2", "split2", "split4"};
  for (int round = 0; round < 2; ++round)
    for (int mode = 0; mode < 6; ++mode)
      printf("{\"probe\": \"%s\", \"round\": %d, \"median_us_per_round_trip\": %.3f}\n", names[mode], round,
             pingpong(req_h, req_d, resp_h, resp_d, 20000, mode, s));
  fflush(stdout);
  {
    std::vector<double> per;
    int d = -1;
    for (int k = 0; k < 22000; ++k) {
      const auto t0 = std::chrono::steady_clock::now();
      for (int j = 0; j < 10; ++j) (void)hipGetDevice(&d);
      if (k >= 2000) per.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / 10);
    }
    std::sort(per.begin(), per.end());
    printf("{\"probe\": \"get_device\", \"median_us\": %.4f}\n", per[per.size() / 2]);
  }
  // the library's C call: one TwoBit pair per call, median of 20000 after 2000 warm calls
  const char* path = getenv("SCTOOLS_HIP_LIB");
  if (!path || !*path) path = "sctools_amd/libsctools_hip.so";
  void* h = dlopen(path, RTLD_NOW);
  if (!h) {
    fprintf(stderr, "dlopen %s: %s\n", path, dlerror());
    return 2;
  }
  auto ham = (hamming_fn)dlsym(h, "sct_hamming_pairs_host");
  auto stop = (stop_fn)dlsym(h, "sct_scalar_server_stop");
  uint64_t a = 0x12345u, b = 0x12344u;
  int32_t out = -1;
  for (int round = 0; round < 2; ++round) {
    std::vector<double> per;
    for (int k = 0; k < 22000; ++k) {
      const auto t0 = std::chrono::steady_clock::now();
      if (ham(2, &a, &b, 1, 1, &out) != 0) return 2;
      if (k >= 2000) per.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    std::sort(per.begin(), per.end());
    printf("{\"probe\": \"c_call\", \"lib\": \"%s\", \"round\": %d, \"median_us\": %.3f, \"p10_us\": %.3f, \"p90_us\": %.3f, "
           "\"out\": %d}\n", path, round, per[per.size() / 2], per[per.size() / 10], per[per.size() * 9 / 10], out);
    fflush(stdout);
  }
  // the other one-record calls: decode (16 bases), gc_content
  {
    auto dec = (decode2_fn)dlsym(h, "sct_decode2_host");
    auto gcf = (gc_fn)dlsym(h, "sct_gc_content_host");
    uint8_t o64[64];
    int32_t g = 0;
    const int Ls[6] = {16, 1, 4, 8, 32, 16};
    for (int which = 0; which < 7; ++which) {
      const int L = which < 6 ? Ls[which] : 16;
      std::vector<double> per;
      for (int k = 0; k < 12000; ++k) {
        const auto t0 = std::chrono::steady_clock::now();
        const int rc = which < 6 ? dec(&a, 1, 1, L, o64) : gcf(2, &a, 1, 1, 16, &g);
        if (rc != 0) return 2;
        if (k >= 2000) per.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
      }
      std::sort(per.begin(), per.end());
      printf("{\"probe\": \"%s\", \"L\": %d, \"median_us\": %.3f, \"p90_us\": %.3f}\n", which < 6 ? "c_decode2" : "c_gc",
             L, per[per.size() / 2], per[per.size() * 9 / 10]);
    }
  }
  // the same call after d ns of host work between calls (the Python wrapper's share), d = 0..2000:
  // a polled mailbox answers in steps of the poll period, so the latency depends on the phase
  for (int d = 0; d <= 2000; d += 100) {
    std::vector<double> per;
    for (int k = 0; k < 3500; ++k) {
      const auto w0 = std::chrono::steady_clock::now();
      while (std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - w0).count() < d) {
      }
      const auto t0 = std::chrono::steady_clock::now();
      if (ham(2, &a, &b, 1, 1, &out) != 0) return 2;
      if (k >= 500) per.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    std::sort(per.begin(), per.end());
    printf("{\"probe\": \"c_call_after_host_work\", \"host_ns\": %d, \"median_us\": %.3f, \"p90_us\": %.3f}\n", d,
           per[per.size() / 2], per[per.size() * 9 / 10]);
  }
  fflush(stdout);
  stop();
  (void)hipHostFree(req_h);
  (void)hipHostFree(resp_h);
  return 0;
}
