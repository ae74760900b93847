// Probe of v_mfma_f32_32x32x16_bf16 lane layouts on gfx950 (tooling, not product).
// A[m][k] = m*16 + k (as bf16-exact small ints scaled), B = identity-like to read back mapping.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void probe(const float* A, const float* B, float* C, int* meta) {
  const int l = threadIdx.x;
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) {
    // hypothesis: A lane l holds A[l%32][8*(l/32)+i], B lane l holds B[8*(l/32)+i][l%32]
    a[i] = (__bf16)A[(l % 32) * 16 + 8 * (l / 32) + i];
    b[i] = (__bf16)B[(8 * (l / 32) + i) * 32 + (l % 32)];
  }
  f32x16 c = {};
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  for (int r = 0; r < 16; ++r) C[l * 16 + r] = c[r];
}

int main() {
  float hA[32 * 16], hB[16 * 32], hC[64 * 16];
  for (int m = 0; m < 32; ++m) for (int k = 0; k < 16; ++k) hA[m * 16 + k] = (k == 0) ? (float)m : 0.f;  // A[m][0] = m
  for (int k = 0; k < 16; ++k) for (int n = 0; n < 32; ++n) hB[k * 32 + n] = (k == 0) ? 1.f : 0.f;     // B[0][n] = 1
  // C[m][n] = m for all n: reveals the row index of each register
  float *dA, *dB, *dC; int* dm;
  hipMalloc(&dA, sizeof hA); hipMalloc(&dB, sizeof hB); hipMalloc(&dC, sizeof hC); hipMalloc(&dm, 4);
  hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice); hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dC, dm);
  hipMemcpy(hC, dC, sizeof hC, hipMemcpyDeviceToHost);
  int ok = 1;
  for (int l = 0; l < 64; ++l) for (int r = 0; r < 16; ++r) {
    int want = 8 * (r / 4) + 4 * (l / 32) + (r % 4);
    if ((int)hC[l * 16 + r] != want) { ok = 0; if (l < 2) printf("lane %d r %d got %g want %d\n", l, r, hC[l * 16 + r], want); }
  }
  // column test: B[0][n] = n, A[m][0] = 1 -> C[m][n] = n; hypothesis n = l % 32
  for (int m = 0; m < 32; ++m) for (int k = 0; k < 16; ++k) hA[m * 16 + k] = (k == 0) ? 1.f : 0.f;
  for (int k = 0; k < 16; ++k) for (int n = 0; n < 32; ++n) hB[k * 32 + n] = (k == 0) ? (float)n : 0.f;
  hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice); hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dC, dm);
  hipMemcpy(hC, dC, sizeof hC, hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) for (int r = 0; r < 16; ++r) if ((int)hC[l * 16 + r] != l % 32) { ok = 0; }
  // k-index test: A[m][k] = 1 for k == 9, B[k][n] = 1 for k == 9 -> all C = 1 iff both map k=9 consistently
  for (int m = 0; m < 32; ++m) for (int k = 0; k < 16; ++k) hA[m * 16 + k] = (k == 9) ? 1.f : 0.f;
  for (int k = 0; k < 16; ++k) for (int n = 0; n < 32; ++n) hB[k * 32 + n] = (k == 9) ? 2.f : 0.f;
  hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice); hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dC, dm);
  hipMemcpy(hC, dC, sizeof hC, hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) for (int r = 0; r < 16; ++r) if (hC[l * 16 + r] != 2.f) { ok = 0; }
  printf("layout hypothesis %s\n", ok ? "CONFIRMED" : "WRONG");
  return ok ? 0 : 1;
}
