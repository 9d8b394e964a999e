// Tile-shape bandwidth probe (development tool): each workgroup stages a
// ROWS x BYTES window of a 1241-stride image batch into LDS (branch-free dword
// loads) and writes an output tile of OROWS x OBYTES to a 1152-pitch batch.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int ROWS, int BYTES, int OROWS, int OBYTES, bool WRITE>
__global__ __launch_bounds__(256) void tile_rw(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                               int tilesX, int tilesY, size_t imgIn, size_t imgOut) {
  constexpr int DW = BYTES / 4, N = ROWS * DW, PER = (N + 255) / 256;
  __shared__ uint32_t t[N];
  const int tile = blockIdx.x, img = blockIdx.y;
  const int ty = tile / tilesX, tx = tile - ty * tilesX;
  const uint8_t* base = src + img * imgIn + (size_t)(ty * OROWS) * 1241 + tx * OBYTES;
  uint32_t lo[PER], hi[PER], sh[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int i = min(q * 256 + (int)threadIdx.x, N - 1);
    const int r = i / DW, k = i - r * DW;
    const uint8_t* p = base + (size_t)r * 1241 + 4 * k;
    sh[q] = (uintptr_t)p & 3;
    const uint32_t* a = (const uint32_t*)(p - sh[q]);
    lo[q] = a[0];
    hi[q] = a[1];
  }
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int i = q * 256 + threadIdx.x;
    if (i < N) t[i] = __builtin_amdgcn_alignbyte(hi[q], lo[q], sh[q]);
  }
  __syncthreads();
  if (WRITE) {
    constexpr int ODW = OBYTES / 4, ON = OROWS * ODW;
    uint8_t* ob = dst + img * imgOut + (size_t)(ty * OROWS) * 1152 + tx * OBYTES;
    for (int i = threadIdx.x; i < ON; i += 256) {
      const int r = i / ODW, k = i - r * ODW;
      *(uint32_t*)(ob + (size_t)r * 1152 + 4 * k) = t[(i * 7) % N] + 1;
    }
  } else if (t[threadIdx.x] == 0x12345678u) {
    dst[0] = 1;
  }
}

int main() {
  const int W = 1241, H = 376, B = 512;
  const size_t imgIn = (size_t)W * H, imgOut = (size_t)1152 * 320;
  uint8_t *a, *b;
  hipMalloc(&a, imgIn * B + 4096);
  hipMalloc(&b, imgOut * B + 4096);
  hipMemset(a, 3, imgIn * B);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](const char* name, double bytes, auto launch) {
    for (int w = 0; w < 3; ++w) launch();
    hipEventRecord(e0);
    for (int it = 0; it < 10; ++it) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%-40s %8.1f GB/s (%.3f ms)\n", name, bytes * 10 / (ms * 1e-3) / 1e9, ms / 10);
  };
#define CASE(R, BY, OR, OB, WR)                                                                  \
  {                                                                                             \
    const int tX = 1030 / OB, tY = 300 / OR;                                                    \
    const double by = (double)B * tX * tY * ((double)R * BY + (WR ? (double)OR * OB : 0.0));   \
    run(#R "x" #BY " -> " #OR "x" #OB " write=" #WR, by, [&] {                                  \
      tile_rw<R, BY, OR, OB, WR><<<dim3(tX * tY, B), 256>>>(a, b, tX, tY, imgIn, imgOut);       \
    });                                                                                         \
  }
  CASE(42, 168, 32, 128, false)
  CASE(42, 168, 32, 128, true)
  CASE(82, 168, 64, 128, true)
  CASE(22, 328, 16, 256, true)
  CASE(12, 648, 8, 512, true)
  CASE(21, 648, 16, 512, true)
  CASE(11, 1240, 8, 1024, true)
  CASE(42, 168, 32, 128, true)
  return 0;
}
