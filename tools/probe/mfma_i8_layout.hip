// Probe: operand / result lane maps of __builtin_amdgcn_mfma_i32_16x16x64_i8 on
// gfx950, checked with exact integer data against a CPU product.
// Assumed: lane l holds A[l & 15][16 (l >> 4) + j] and B[16 (l >> 4) + j][l & 15]
// (j = 0..15, byte j of its 4 dwords); D: col = l & 15, row = 4 (l >> 4) + i.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
typedef int v4i __attribute__((ext_vector_type(4)));
__global__ void k(const int8_t* A, const int8_t* B, int32_t* D) {
  const int l = threadIdx.x;
  v4i a, b;
  int8_t* ab = (int8_t*)&a;
  int8_t* bb = (int8_t*)&b;
  for (int j = 0; j < 16; ++j) {
    ab[j] = A[(l & 15) * 64 + 16 * (l >> 4) + j];
    bb[j] = B[(16 * (l >> 4) + j) * 16 + (l & 15)];
  }
  v4i c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
  for (int i = 0; i < 4; ++i) D[(4 * (l >> 4) + i) * 16 + (l & 15)] = c[i];
}
int main() {
  int8_t hA[16 * 64], hB[64 * 16];
  int32_t hD[256], ref[256];
  srand(7);
  for (int i = 0; i < 16 * 64; ++i) hA[i] = (int8_t)(rand() % 256 - 128);
  for (int i = 0; i < 64 * 16; ++i) hB[i] = (int8_t)(rand() % 256 - 128);
  for (int r = 0; r < 16; ++r)
    for (int c = 0; c < 16; ++c) {
      int s = 0;
      for (int k = 0; k < 64; ++k) s += hA[r * 64 + k] * hB[k * 16 + c];
      ref[r * 16 + c] = s;
    }
  int8_t *dA, *dB;
  int32_t* dD;
  hipMalloc(&dA, sizeof hA); hipMalloc(&dB, sizeof hB); hipMalloc(&dD, sizeof hD);
  hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 256; ++i) bad += hD[i] != ref[i];
  printf("mfma_i32_16x16x64_i8 layout: %d of 256 mismatches\n", bad);
  return bad != 0;
}
