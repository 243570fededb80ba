// VALU issue rate vs VGPR bank pattern on gfx950: blocks of hand-placed instructions
// with fixed registers (v32..v79), no dependencies between consecutive instructions.
//   hipcc --offload-arch=gfx950 -O3 tools/valu_banks.hip -o tools/valu_banks
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define STR2(x) #x
#define STR(x) STR2(x)

// 16 instructions per block; destinations v32..v47 (banks rotate), sources per pattern
#define BLK16(OP)                                                                          \
  OP(32) OP(33) OP(34) OP(35) OP(36) OP(37) OP(38) OP(39) OP(40) OP(41) OP(42) OP(43) OP(44) \
      OP(45) OP(46) OP(47)

// sources in three different banks (b = 48..: 48%4=0, 49%4=1, 50%4=2)
#define B3_DIFF(d) "v_bitop3_b32 v" STR(d) ", v48, v49, v50 bitop3:0x96\n"
// sources all in bank 0
#define B3_SAME(d) "v_bitop3_b32 v" STR(d) ", v48, v52, v56 bitop3:0x96\n"
// two sources same register
#define B3_DUP(d) "v_bitop3_b32 v" STR(d) ", v48, v48, v49 bitop3:0x96\n"
#define B3_TWO01(d) "v_bitop3_b32 v" STR(d) ", v48, v52, v49 bitop3:0x96\n"
#define B3_TWO02(d) "v_bitop3_b32 v" STR(d) ", v48, v49, v52 bitop3:0x96\n"
#define B3_TWO12(d) "v_bitop3_b32 v" STR(d) ", v49, v48, v52 bitop3:0x96\n"
#define MIX_B3_BCNT(d) "v_bitop3_b32 v" STR(d) ", v48, v49, v50 bitop3:0x96\n v_bcnt_u32_b32 v" STR(d) ", v49, v" STR(d) "\n"
#define BCNT_DIFF(d) "v_bcnt_u32_b32 v" STR(d) ", v48, v49\n"
#define BCNT_SAME(d) "v_bcnt_u32_b32 v" STR(d) ", v48, v52\n"
#define BCNT_K(d) "v_bcnt_u32_b32 v" STR(d) ", v48, 0\n"
#define XOR_SAME(d) "v_xor_b32_e64 v" STR(d) ", v48, v52\n"
#define XOR_DIFF(d) "v_xor_b32 v" STR(d) ", v48, v49\n"
#define AND3_DIFF(d) "v_and_or_b32 v" STR(d) ", v48, v49, v50\n"
#define B3_SGPR(d) "v_bitop3_b32 v" STR(d) ", v48, s20, v50 bitop3:0x96\n"

#define CLOB                                                                                    \
  "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", \
      "v46", "v47"

#define KERNEL(NAME, OP)                                                                 \
  __global__ __launch_bounds__(256) void NAME(uint32_t* out, int iters) {                \
    asm volatile("v_mov_b32 v48, %0\n v_mov_b32 v49, %1\n v_mov_b32 v50, %0\n"           \
                 "v_mov_b32 v52, %1\n v_mov_b32 v56, %0\n s_mov_b32 s20, 7\n" ::"v"(threadIdx.x), \
                 "v"(blockIdx.x)                                                         \
                 : "v48", "v49", "v50", "v52", "v56", "s20");                            \
    for (int i = 0; i < iters; ++i) {                                                    \
      asm volatile(BLK16(OP) BLK16(OP) BLK16(OP) BLK16(OP)::: CLOB);                     \
    }                                                                                    \
    uint32_t r;                                                                          \
    asm volatile("v_mov_b32 %0, v40" : "=v"(r));                                         \
    out[blockIdx.x * 256 + threadIdx.x] = r;                                             \
  }

KERNEL(k_b3_diff, B3_DIFF)
KERNEL(k_b3_same, B3_SAME)
KERNEL(k_b3_dup, B3_DUP)
KERNEL(k_b3_two01, B3_TWO01)
KERNEL(k_b3_two02, B3_TWO02)
KERNEL(k_b3_two12, B3_TWO12)
KERNEL(k_mix, MIX_B3_BCNT)
KERNEL(k_bcnt_diff, BCNT_DIFF)
KERNEL(k_bcnt_same, BCNT_SAME)
KERNEL(k_bcnt_k, BCNT_K)
KERNEL(k_xor_same, XOR_SAME)
KERNEL(k_xor_diff, XOR_DIFF)
KERNEL(k_andor_diff, AND3_DIFF)
KERNEL(k_b3_sgpr, B3_SGPR)

typedef void (*kfn)(uint32_t*, int);

static void run(const char* name, kfn f) {
  const int blocks = 256 * 8, iters = 2048;
  uint32_t* out;
  (void)hipMalloc(&out, (size_t)blocks * 256 * 4);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, out, iters);
  (void)hipEventRecord(a);
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, out, iters);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  const double lane_ops = 3.0 * blocks * 256.0 * iters * 64;
  printf("{\"op\": \"%s\", \"ms\": %.3f, \"lane_ops_per_s\": %.4e, \"per_cu_per_clk_at_2.3GHz\": %.1f}\n",
         name, ms / 3, lane_ops / (ms * 1e-3), lane_ops / (ms * 1e-3) / 256 / 2.3e9);
  (void)hipFree(out);
}

int main() {
  run("bitop3 3 banks", k_b3_diff);
  run("bitop3 1 bank", k_b3_same);
  run("bitop3 dup src", k_b3_dup);
  run("bitop3 src0,src1 same bank", k_b3_two01);
  run("bitop3 src0,src2 same bank", k_b3_two02);
  run("bitop3 src1,src2 same bank", k_b3_two12);
  run("bitop3+bcnt pairs (x2 ops)", k_mix);
  run("bitop3 vgpr,sgpr,vgpr", k_b3_sgpr);
  run("bcnt 2 banks", k_bcnt_diff);
  run("bcnt 1 bank", k_bcnt_same);
  run("bcnt vgpr,0", k_bcnt_k);
  run("xor_e64 1 bank", k_xor_same);
  run("xor_e32 2 banks", k_xor_diff);
  run("and_or 3 banks", k_andor_diff);
  return 0;
}
