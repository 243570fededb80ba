// Measured integer-VALU peak on gfx950: throughput of the instructions the all-pairs
// kernel issues (v_bitop3_b32, v_bcnt_u32_b32, v_xor_b32) in long independent
// chains, all CUs busy, plus the in-kernel clock (s_memtime / s_memrealtime).
//   hipcc --offload-arch=gfx950 -O3 tools/valu_peak.hip -o tools/valu_peak && tools/valu_peak
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHK(x)                                                                   \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                     \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

constexpr int ITERS = 4096;
constexpr int CH = 12;  // independent chains per lane

template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t x[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) x[c] = seed * (threadIdx.x + 1) + c * 0x9E3779B9u;
  const uint32_t y = seed ^ threadIdx.x, z = seed + blockIdx.x;
  double dacc[CH];  // OPs 18-20: fp64 accumulate of a square
#pragma unroll
  for (int c = 0; c < CH; ++c) dacc[c] = (double)x[c];
  const double dz = (double)(int)z;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      if constexpr (OP == 0) x[c] = __builtin_amdgcn_bitop3_b32(x[c], y, z, 0x96);
      if constexpr (OP == 1) asm volatile("v_bcnt_u32_b32 %0, %1, %0" : "+v"(x[c]) : "v"(y));
      if constexpr (OP == 2) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(x[c]) : "v"(y));
      if constexpr (OP == 4) asm volatile("v_xor_b32_e64 %0, %1, %0" : "+v"(x[c]) : "v"(y));
      if constexpr (OP == 5) asm volatile("v_add3_u32 %0, %1, %2, %0" : "+v"(x[c]) : "v"(y), "v"(z));
      if constexpr (OP == 6) asm volatile("v_or3_b32 %0, %1, %2, %0" : "+v"(x[c]) : "v"(y), "v"(z));
      if constexpr (OP == 7) {  // alternate 8-byte and 4-byte encodings
        asm volatile("v_bcnt_u32_b32 %0, %1, %0" : "+v"(x[c]) : "v"(y));
        asm volatile("v_xor_b32 %0, %1, %0" : "+v"(x[c]) : "v"(z));
      }
      if constexpr (OP == 8) asm volatile("v_add_u32 %0, %1, %0" : "+v"(x[c]) : "v"(y));
      if constexpr (OP == 9) asm volatile("v_and_b32 %0, %1, %0" : "+v"(x[c]) : "v"(y));
      if constexpr (OP == 10) {  // 64-bit accumulate of a square: v_mad_i64_i32
        uint64_t a64 = ((uint64_t)x[c] << 32) | y;
        asm volatile("v_mad_i64_i32 %0, vcc, %1, %1, %0" : "+v"(a64) : "v"(z) : "vcc");
        x[c] = (uint32_t)a64 ^ (uint32_t)(a64 >> 32);
      }
      if constexpr (OP == 11) asm volatile("v_mul_i32_i24 %0, %1, %0" : "+v"(x[c]) : "v"(y));
      if constexpr (OP == 12) asm volatile("v_mul_hi_i32_i24 %0, %1, %0" : "+v"(x[c]) : "v"(y));
      if constexpr (OP == 13) asm volatile("v_lshl_add_u32 %0, %1, 8, %0" : "+v"(x[c]) : "v"(y));
      if constexpr (OP == 14) asm volatile("v_perm_b32 %0, %1, %0, %2" : "+v"(x[c]) : "v"(y), "v"(z));
      if constexpr (OP == 15) asm volatile("v_pk_add_u16 %0, %1, %0" : "+v"(x[c]) : "v"(y));
      if constexpr (OP == 16) asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(x[c]) : "v"(y), "v"(z));
      if constexpr (OP == 17) asm volatile("v_mul_lo_u32 %0, %1, %0" : "+v"(x[c]) : "v"(y));
      if constexpr (OP == 18) asm volatile("v_fma_f64 %0, %1, %1, %0" : "+v"(dacc[c]) : "v"(dz));
      if constexpr (OP == 19) {  // int32 -> f64, then acc += v * v
        double t;
        asm volatile("v_cvt_f64_i32 %0, %1" : "=v"(t) : "v"(x[c]));
        asm volatile("v_fma_f64 %0, %1, %1, %0" : "+v"(dacc[c]) : "v"(t));
      }
      if constexpr (OP == 20) {
        double t;
        asm volatile("v_cvt_f64_i32 %0, %1" : "=v"(t) : "v"(x[c]));
        x[c] ^= (uint32_t)__builtin_bit_cast(uint64_t, t);
      }
      if constexpr (OP == 21) {  // packed int16 dot: acc += a.lo * b.lo + a.hi * b.hi
        typedef short s2 __attribute__((ext_vector_type(2)));
        x[c] = (uint32_t)__builtin_amdgcn_sdot2(__builtin_bit_cast(s2, y), __builtin_bit_cast(s2, z), (int)x[c], false);
      }
      if constexpr (OP == 3) {  // the kernel's mix: 2 bitop3 : 1 bcnt
        x[c] = __builtin_amdgcn_bitop3_b32(x[c], y, z, 0xE8);
        x[c] = __builtin_amdgcn_bitop3_b32(x[c], y, z, 0x96);
        asm volatile("v_bcnt_u32_b32 %0, %1, %0" : "+v"(x[c]) : "v"(y));
      }
    }
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint64_t r1 = __builtin_amdgcn_s_memrealtime();
  uint32_t acc = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) acc ^= x[c] ^ (uint32_t)__builtin_bit_cast(uint64_t, dacc[c]);
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

template <int OP>
int run(const char* name, int ops_per_chain_iter, int blocks) {
  uint32_t* out;
  uint64_t* clk;
  CHK(hipMalloc(&out, (size_t)blocks * 256 * 4));
  CHK(hipMalloc(&clk, (size_t)blocks * 16));
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, clk, 7u);
  CHK(hipEventRecord(a));
  const int reps = 5;
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, clk, 7u + r);
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, a, b));
  uint64_t* h = new uint64_t[2 * blocks];
  CHK(hipMemcpy(h, clk, (size_t)blocks * 16, hipMemcpyDeviceToHost));
  double ratio = 0;
  for (int i = 0; i < blocks; ++i) ratio += (double)h[2 * i] / (double)h[2 * i + 1];
  const double ghz = ratio / blocks * 0.1;  // s_memrealtime ticks at 100 MHz
  const double lane_ops = (double)reps * blocks * 256.0 * ITERS * CH * ops_per_chain_iter;
  const double ops_s = lane_ops / (ms * 1e-3);
  printf("{\"op\": \"%s\", \"blocks\": %d, \"ms\": %.3f, \"lane_ops_per_s\": %.4e, \"clock_ghz\": %.3f, "
         "\"lane_ops_per_clk_per_cu\": %.2f}\n",
         name, blocks, ms / reps, ops_s, ghz, ops_s / (ghz * 1e9) / 256.0);
  delete[] h;
  (void)hipFree(out);
  (void)hipFree(clk);
  return 0;
}

int main() {
  const int blocks = 256 * 8;  // 8 workgroups (32 waves) per CU
  run<0>("v_bitop3_b32", 1, blocks);
  run<1>("v_bcnt_u32_b32", 1, blocks);
  run<2>("v_xor_b32", 1, blocks);
  run<3>("mix_2bitop3_1bcnt", 3, blocks);
  run<0>("v_bitop3_b32@2wps", 1, 256 * 2);
  run<4>("v_xor_b32_e64", 1, blocks);
  run<5>("v_add3_u32", 1, blocks);
  run<6>("v_or3_b32", 1, blocks);
  run<7>("bcnt+xor_e32", 2, blocks);
  run<8>("v_add_u32_e32", 1, blocks);
  run<9>("v_and_b32_e32", 1, blocks);
  run<10>("v_mad_i64_i32(+2 xor/shift)", 1, blocks);
  run<11>("v_mul_i32_i24", 1, blocks);
  run<12>("v_mul_hi_i32_i24", 1, blocks);
  run<13>("v_lshl_add_u32", 1, blocks);
  run<14>("v_perm_b32", 1, blocks);
  run<15>("v_pk_add_u16", 1, blocks);
  run<16>("v_mad_u32_u24", 1, blocks);
  run<17>("v_mul_lo_u32", 1, blocks);
  run<18>("v_fma_f64", 1, blocks);
  run<19>("v_cvt_f64_i32+v_fma_f64", 2, blocks);
  run<20>("v_cvt_f64_i32(+xor)", 1, blocks);
  run<21>("v_dot2_i32_i16", 1, blocks);
  run<2>("v_xor_b32@1wps", 1, 256);
  run<2>("v_xor_b32@2wps", 1, 512);
  run<2>("v_xor_b32@4wps", 1, 1024);
  return 0;
}
