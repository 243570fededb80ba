// Probe the lane -> (row, k) map of v_mfma_i32_16x16x64_i8 operands on gfx950:
// A = one-hot rows, B = distinct small integers; prints where each B element lands.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef long v2l __attribute__((ext_vector_type(2)));

__global__ void probe(const signed char* A, const signed char* B, int* C) {
  const int l = threadIdx.x;
  v4i a, b;
  for (int q = 0; q < 4; ++q) {
    int wa = 0, wb = 0;
    for (int r = 0; r < 4; ++r) {
      wa |= (A[l * 16 + q * 4 + r] & 255) << (8 * r);
      wb |= (B[l * 16 + q * 4 + r] & 255) << (8 * r);
    }
    a[q] = wa;
    b[q] = wb;
  }
  v4i c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_i32_16x16x64_i8(*reinterpret_cast<v2l*>(&a) , *reinterpret_cast<v2l*>(&b), c, 0, 0, 0);
  for (int i = 0; i < 4; ++i) C[l * 4 + i] = c[i];
}

int main() {
  // hypothesis: lane l holds A[m = l & 15][k = 16 (l >> 4) + j], B[k = 16 (l >> 4) + j][n = l & 15]
  signed char hA[64 * 16], hB[64 * 16];
  // A = identity-like: A[m][k] = 1 iff k == m + 16*(m&3)? use A[m][k] = (k == 4*m + 1) to test
  for (int l = 0; l < 64; ++l)
    for (int j = 0; j < 16; ++j) {
      const int m = l & 15, k = 16 * (l >> 4) + j, n = l & 15;
      hA[l * 16 + j] = (k == 4 * m + 1) ? 1 : 0;
      hB[l * 16 + j] = (signed char)((k * 3 + n * 7) % 101);  // B[k][n] (hypothesis map)
    }
  signed char *dA, *dB;
  int* dC;
  hipMalloc(&dA, sizeof hA);
  hipMalloc(&dB, sizeof hB);
  hipMalloc(&dC, 64 * 4 * 4);
  hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dC);
  int hC[256];
  hipMemcpy(hC, dC, sizeof hC, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int i = 0; i < 4; ++i) {
      const int m = 4 * (l >> 4) + i, n = l & 15;  // C map: col = lane & 15, row = 4 (lane >> 4) + reg
      const int want = ((4 * m + 1) * 3 + n * 7) % 101;
      if (hC[l * 4 + i] != want) {
        if (bad < 8) printf("lane %d reg %d: got %d want %d\n", l, i, hC[l * 4 + i], want);
        ++bad;
      }
    }
  printf("mismatches: %d (hypothesis k = 16 (l >> 4) + j %s)\n", bad, bad ? "WRONG" : "holds");
  return bad ? 1 : 0;
}
