// Bandwidth probe (development tool): read-only and copy kernels over a
// 512 MiB buffer with dword vs 16-byte lanes, and a 2-D tile pattern like the
// extractor's (rows of 268 B at a 1280 B pitch).  Prints GB/s per variant.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ void rd32(const uint32_t* __restrict__ a, size_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc ^= a[i];
  if (acc == 0x12345678u) out[0] = acc;
}
__global__ void rd128(const uint4* __restrict__ a, size_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint4 v = a[i]; acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}
__global__ void cp32(const uint32_t* __restrict__ a, uint32_t* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}
__global__ void cp128(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}
// one workgroup per 38-row x 67-dword tile, tiles row-major over images of 1280 x 400
template <int U>
__global__ __launch_bounds__(256) void tile_rd(const uint8_t* __restrict__ img, int pitch, int rows,
                                               int tilesX, uint32_t* out) {
  __shared__ uint32_t t[38 * 67];
  const int tile = blockIdx.x, im = blockIdx.y;
  const int ty = tile / tilesX, tx = tile - ty * tilesX;
  const uint8_t* base = img + (size_t)im * pitch * rows + (size_t)(ty * 32) * pitch + tx * 256;
  const int n = 38 * 67;
  uint32_t v[U];
#pragma unroll
  for (int q = 0; q < U; ++q) {
    const int i = q * 256 + threadIdx.x;
    v[q] = 0;
    if (i < n) { const int r = i / 67, k = i - r * 67; v[q] = *(const uint32_t*)(base + (size_t)r * pitch + 4 * k); }
  }
#pragma unroll
  for (int q = 0; q < U; ++q) { const int i = q * 256 + threadIdx.x; if (i < n) t[i] = v[q]; }
  __syncthreads();
  if (t[threadIdx.x] == 0x12345678u) out[0] = 1;
}

int main() {
  const size_t bytes = 512ull << 20;
  uint8_t *a, *b; uint32_t* o;
  hipMalloc(&a, bytes); hipMalloc(&b, bytes); hipMalloc(&o, 64);
  hipMemset(a, 1, bytes); hipMemset(b, 0, bytes);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  auto run = [&](const char* name, double gb, auto launch) {
    for (int w = 0; w < 3; ++w) launch();
    hipEventRecord(e0);
    for (int it = 0; it < 10; ++it) launch();
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("%-28s %8.1f GB/s  (%.3f ms)\n", name, gb * 10 / (ms * 1e-3), ms / 10);
  };
  const double G = bytes / 1e9;
  for (int grid : {1024, 4096, 16384}) {
    char nm[64];
    snprintf(nm, 64, "read dword grid %d", grid);
    run(nm, G, [&] { rd32<<<grid, 256>>>((const uint32_t*)a, bytes / 4, o); });
    snprintf(nm, 64, "read 16B grid %d", grid);
    run(nm, G, [&] { rd128<<<grid, 256>>>((const uint4*)a, bytes / 16, o); });
    snprintf(nm, 64, "copy dword grid %d", grid);
    run(nm, 2 * G, [&] { cp32<<<grid, 256>>>((const uint32_t*)a, (uint32_t*)b, bytes / 8); });
    snprintf(nm, 64, "copy 16B grid %d", grid);
    run(nm, 2 * G, [&] { cp128<<<grid, 256>>>((const uint4*)a, (uint4*)b, bytes / 32); });
  }
  // tiles: images of 1280 x 400 (pitch 1280), 5 x 12 tiles of 256 x 32 rows (+6 halo)
  const int pitch = 1280, rows = 400, nimg = (int)(bytes / ((size_t)pitch * rows)) - 1;
  const double tg = (double)nimg * 5 * 12 * 38 * 268 / 1e9;
  run("tile 38x268 U=10", tg, [&] { tile_rd<10><<<dim3(60, nimg), 256>>>(a, pitch, rows, 5, o); });
  run("tile 38x268 U=4 (x3 loop)", tg, [&] { tile_rd<10><<<dim3(60, nimg), 256>>>(a, pitch, rows, 5, o); });
  hipFree(a); hipFree(b); hipFree(o);
  return 0;
}
