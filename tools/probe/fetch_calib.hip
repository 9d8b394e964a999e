// FETCH_SIZE / WRITE_SIZE calibration (development probe): rocprofv3 --pmc FETCH_SIZE over
// kernels that each read a known, disjoint 1 GiB once, with the load shapes
// the extractor uses.  MI355X_MICROARCH.md: FETCH_SIZE reports half the bytes
// of 16-B/lane coalesced streaming reads and is uncalibrated for other widths.
//   rd32       dword per lane, consecutive lanes consecutive dwords (resize, blur staging)
//   rd128      16 B per lane, consecutive lanes consecutive 16 B (the guide's case)
//   row64      64 B per lane (four 16-B loads), lane = row of a 1 KiB-pitch
//              image: k_fast_cells' ROI staging (one row per lane), 64-B aligned
//   row64u     the same starting 4 bytes past alignment (caller strides)
//   wr32 / wr128  dword / 16-B stores, coalesced (WRITE_SIZE)
// Run: rocprofv3 --pmc FETCH_SIZE (or WRITE_SIZE) -d <dir> -o run --output-format csv -- tools/probe/fetch_calib
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

__global__ void rd32(const uint32_t* __restrict__ a, size_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    acc ^= a[i];
  if (acc == 0x12345678u) out[0] = acc;
}
__global__ void rd128(const uint4* __restrict__ a, size_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = a[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}
__global__ void wr32(uint32_t* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[i] = (uint32_t)i;
}
__global__ void wr128(uint4* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[i] = make_uint4((uint32_t)i, 0u, 1u, 2u);
}
// image: rows x 1024 B; lane (row r, window j) reads bytes [r*1024 + 64 j + s, +64)
__global__ void row64(const uint8_t* __restrict__ img, int rows, int s, uint32_t* out) {
  const int lane = threadIdx.x & 63;
  const int w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;  // wave
  const int rowsPerWave = 64;
  const int r = (w / 16) * rowsPerWave + lane, j = w % 16;
  if (r >= rows) return;
  const uint8_t* base = img + (size_t)(r / 1024) * 1024 * 1024;  // 1 MiB slabs: 32-bit offsets
  const __amdgpu_buffer_rsrc_t rs = rsrc(base, 1024 * 1024 + 64);
  const uint32_t o = (uint32_t)((r % 1024) * 1024 + 64 * j + s);
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(o + 16 * k), 0, 0);
    acc ^= (uint32_t)v[0] ^ (uint32_t)v[1] ^ (uint32_t)v[2] ^ (uint32_t)v[3];
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  const size_t bytes = 1ull << 30;
  uint8_t* a;
  uint32_t* o;
  if (hipMalloc(&a, bytes + 4096) != hipSuccess || hipMalloc(&o, 64) != hipSuccess) return 1;
  hipMemset(a, 1, bytes + 4096);
  hipDeviceSynchronize();
  hipLaunchKernelGGL(rd32, dim3(8192), dim3(256), 0, 0, (const uint32_t*)a, bytes / 4, o);
  hipLaunchKernelGGL(rd128, dim3(8192), dim3(256), 0, 0, (const uint4*)a, bytes / 16, o);
  const int rows = (int)(bytes / 1024);
  const int waves = rows / 64 * 16;
  hipLaunchKernelGGL(row64, dim3(waves / 4), dim3(256), 0, 0, a, rows, 0, o);
  hipLaunchKernelGGL(row64, dim3(waves / 4), dim3(256), 0, 0, a, rows, 4, o);
  hipLaunchKernelGGL(wr32, dim3(8192), dim3(256), 0, 0, (uint32_t*)a, bytes / 4);
  hipLaunchKernelGGL(wr128, dim3(8192), dim3(256), 0, 0, (uint4*)a, bytes / 16);
  hipDeviceSynchronize();
  printf("each kernel reads (rd*, row64) or writes (wr*)  %zu bytes once (row64 with s=4 reads 4 bytes past the end of its last row)\n", bytes);
  return 0;
}
