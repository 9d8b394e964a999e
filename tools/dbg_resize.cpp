// Debug harness: one k_pyr_resize launch vs the oracle resize (dev tool).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
#include <algorithm>
extern "C" hipError_t orb_k_pyr_resize(const uint8_t* src, long long srcImgPitch, int srcStride, int sw, int sh,
                            uint8_t* dst, long long dstImgPitch, int dstStride, int dw, int dh,
                            const int* xofs, const void* alpha, const int* yofs, const void* beta,
                            int xmax, int nimg, hipStream_t s);
extern "C" int oracle_resize(const uint8_t* src, int sw, int sh, uint8_t* dst, int dw, int dh);
extern "C" void oracle_synth_image(uint64_t seed, int frame, int view, int w, int h, uint8_t* out, size_t stride);
int main() {
  int sw = 640, sh = 480, dw = 533, dh = 400;
  std::vector<uint8_t> img(sw * sh), ref(dw * dh), got(dw * dh);
  oracle_synth_image(1, 0, 0, sw, sh, img.data(), sw);
  oracle_resize(img.data(), sw, sh, ref.data(), dw, dh);
  std::vector<int> rt(2 * dw + 2 * dh);
  double scale_x = 1. / ((double)dw / sw), scale_y = 1. / ((double)dh / sh);
  int xmax = dw;
  for (int dx = 0; dx < dw; ++dx) {
    float fx = (float)((dx + 0.5) * scale_x - 0.5); int sx = (int)floorf(fx); fx -= sx;
    if (sx < 0) { fx = 0; sx = 0; }
    if (sx + 1 >= sw) { xmax = std::min(xmax, dx); if (sx >= sw - 1) { fx = 0; sx = sw - 1; } }
    short a0 = (short)lrintf((1.f - fx) * 2048), a1 = (short)lrintf(fx * 2048);
    rt[dx] = sx; rt[dw + dx] = (int)(((uint32_t)(uint16_t)a1 << 16) | (uint16_t)a0);
  }
  for (int dy = 0; dy < dh; ++dy) {
    float fy = (float)((dy + 0.5) * scale_y - 0.5); int sy = (int)floorf(fy); fy -= sy;
    short b0 = (short)lrintf((1.f - fy) * 2048), b1 = (short)lrintf(fy * 2048);
    rt[2 * dw + dy] = sy; rt[2 * dw + dh + dy] = (int)(((uint32_t)(uint16_t)b1 << 16) | (uint16_t)b0);
  }
  uint8_t *dsrc, *ddst; int* drt;
  hipMalloc(&dsrc, sw * sh); hipMalloc(&ddst, 576 * dh); hipMalloc(&drt, rt.size() * 4);
  hipMemcpy(dsrc, img.data(), sw * sh, hipMemcpyHostToDevice);
  hipMemcpy(drt, rt.data(), rt.size() * 4, hipMemcpyHostToDevice);
  hipMemset(ddst, 0, 576 * dh);
  hipError_t e = orb_k_pyr_resize(dsrc, sw * sh, sw, sw, sh, ddst, 576 * dh, 576, dw, dh, drt, drt + dw, drt + 2 * dw, drt + 2 * dw + dh, xmax, 1, 0);
  hipDeviceSynchronize();
  hipMemcpy2D(got.data(), dw, ddst, 576, dw, dh, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < dw * dh; ++i) bad += got[i] != ref[i];
  printf("launch %d, mismatches %d of %d\n", (int)e, bad, dw * dh);
  for (int x = 0; x < 12; ++x) printf("%d/%d ", got[x], ref[x]);
  printf("\n");
  return 0;
}
