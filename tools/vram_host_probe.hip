// Can the host write device memory directly (a large-BAR mapping), so the scalar server could poll
// a request line in its own HBM instead of reading host memory over PCIe?
// For each allocation kind: the runtime's pointer attributes (a host address, if any), and -- only
// when the runtime reports one -- a host write, a kernel that reads it back and writes an answer,
// and the round-trip latency of that ping-pong against the same loop on host-coherent memory.
//   hipcc --offload-arch=gfx950 -O2 tools/vram_host_probe.hip -o tools/vram_host_probe && tools/vram_host_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <chrono>

#define CHK(x)                                                                   \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                     \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

// one lane polls req[0] for a new sequence number and echoes it into resp[0]; exits on seq < 0
__global__ void ping(volatile int* req, volatile int* resp, int rounds) {
  if (threadIdx.x != 0) return;
  int last = 0;
  for (int r = 0; r < rounds; ++r) {
    int v;
    uint64_t spins = 0;
    do {
      v = __hip_atomic_load(req, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
      if (++spins > (1ull << 28)) return;  // (never wait forever)
    } while (v == last);
    last = v;
    __hip_atomic_store(resp, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

static double pingpong(volatile int* req_host, int* req_dev, volatile int* resp_host, int* resp_dev, int rounds) {
  *req_host = 0;
  *resp_host = 0;
  hipLaunchKernelGGL(ping, dim3(1), dim3(64), 0, 0, req_dev, resp_dev, rounds);
  auto t0 = std::chrono::steady_clock::now();
  for (int r = 1; r <= rounds; ++r) {
    __atomic_store_n(req_host, r, __ATOMIC_RELEASE);
    uint64_t spins = 0;
    while (__atomic_load_n(resp_host, __ATOMIC_ACQUIRE) != r)
      if (++spins > (1ull << 32)) return -1.0;
  }
  auto t1 = std::chrono::steady_clock::now();
  (void)hipDeviceSynchronize();
  return std::chrono::duration<double, std::micro>(t1 - t0).count() / rounds;
}

int main() {
  int* resp_h = nullptr;
  int* resp_d = nullptr;
  CHK(hipHostMalloc((void**)&resp_h, 4096, hipHostMallocCoherent | hipHostMallocMapped));
  CHK(hipHostGetDevicePointer((void**)&resp_d, resp_h, 0));
  // baseline: request line in host-coherent memory (what the scalar server does today)
  {
    int* req_h = nullptr;
    int* req_d = nullptr;
    CHK(hipHostMalloc((void**)&req_h, 4096, hipHostMallocCoherent | hipHostMallocMapped));
    CHK(hipHostGetDevicePointer((void**)&req_d, req_h, 0));
    printf("{\"kind\": \"host_coherent\", \"us_per_round_trip\": %.3f}\n", pingpong(req_h, req_d, resp_h, resp_d, 20000));
    (void)hipHostFree(req_h);
  }
  struct Kind {
    const char* name;
    unsigned flags;
  } kinds[] = {{"hipDeviceMallocDefault", hipDeviceMallocDefault},
               {"hipDeviceMallocFinegrained", hipDeviceMallocFinegrained},
               {"hipDeviceMallocUncached", hipDeviceMallocUncached}};
  for (const Kind& k : kinds) {
    void* p = nullptr;
    hipError_t e = hipExtMallocWithFlags(&p, 4096, k.flags);
    if (e != hipSuccess) {
      printf("{\"kind\": \"%s\", \"alloc\": \"%s\"}\n", k.name, hipGetErrorString(e));
      (void)hipGetLastError();
      continue;
    }
    hipPointerAttribute_t a{};
    e = hipPointerGetAttributes(&a, p);
    void* hp = e == hipSuccess ? a.hostPointer : nullptr;
    printf("{\"kind\": \"%s\", \"attr\": \"%s\", \"type\": %d, \"devicePointer\": \"%p\", \"hostPointer\": \"%p\"",
           k.name, hipGetErrorString(e), (int)a.type, a.devicePointer, hp);
    if (hp) {
      printf(", \"us_per_round_trip\": %.3f", pingpong((volatile int*)hp, (int*)p, resp_h, resp_d, 20000));
    }
    printf("}\n");
    fflush(stdout);
    (void)hipFree(p);
  }
  (void)hipHostFree(resp_h);
  return 0;
}
