// C++ host mirror smoke/parity test (tests/test_cpp_host.py builds and runs it).
// ORB_SLAM2-style calls through orb_amd.hpp, checked against the CPU oracle's
// C entry points (test infrastructure).
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../orb_slam2-chinese-annotation_amd/host/orb_amd.hpp"

extern "C" int oracle_extract(const uint8_t* img, int w, int h, size_t stride, int nfeatures,
                              float scaleFactor, int nlevels, int iniTh, int minTh,
                              orb_keypoint_t* kps, uint8_t* desc, int cap, int32_t* per_level);
extern "C" int oracle_match_projection_local(const orb_frame_t* F, const uint8_t* kp_locked,
                                             int nmp, const orb_mp_track_t* mps,
                                             const uint8_t* mp_desc, float th, float nnratio,
                                             int32_t* kp_match);

int main() {
  const int W = 1241, H = 376;
  std::vector<uint8_t> img((size_t)W * H);
  orb_synth_image(77, 0, 0, W, H, img.data(), W);
  orb_amd::ORBextractor extractor(1000, 1.2f, 8, 20, 7);
  std::vector<orb_amd::KeyPoint> kps;
  orb_amd::Descriptors desc;
  extractor({img.data(), W, H, (size_t)W}, {}, kps, desc);

  std::vector<orb_keypoint_t> rk(4000);
  std::vector<uint8_t> rd(4000 * 32);
  const int n = oracle_extract(img.data(), W, H, W, 1000, 1.2f, 8, 20, 7, rk.data(), rd.data(),
                               4000, nullptr);
  if (n != (int)kps.size() || memcmp(rk.data(), kps.data(), n * sizeof(orb_keypoint_t)) ||
      memcmp(rd.data(), desc.data.data(), (size_t)n * 32)) {
    printf("FAIL extract: gpu %zu oracle %d\n", kps.size(), n);
    return 1;
  }
  // empty image: outputs untouched (src/ORBextractor.cc:1095-1096)
  extractor({nullptr, 0, 0, 0}, {}, kps, desc);
  if ((int)kps.size() != n) { printf("FAIL empty image touched outputs\n"); return 1; }

  orb_amd::FrameView F;
  F.mvKeysUn = kps;
  F.mDescriptors = desc;
  F.mnMaxX = (float)W;
  F.mnMaxY = (float)H;
  F.mvScaleFactors = extractor.GetScaleFactors();
  const int M = 5000;
  std::vector<orb_mp_track_t> mps(M);
  std::vector<uint8_t> mpd((size_t)M * 32), locked(n);
  orb_synth_local_map(77, kps.data(), desc.data.data(), n, M, W, H, mps.data(), mpd.data(),
                      locked.data());
  orb_amd::ORBmatcher matcher(0.8f);
  std::vector<int32_t> mvp(n, -1);
  const int nm = matcher.SearchByProjection(F, mps, mpd, 1.0f, mvp, locked);
  const orb_frame_t fc = F.c();
  std::vector<int32_t> ref(n, -1);
  const int nr = oracle_match_projection_local(&fc, locked.data(), M, mps.data(), mpd.data(), 1.0f,
                                               0.8f, ref.data());
  if (nm != nr || mvp != ref) { printf("FAIL match: gpu %d oracle %d\n", nm, nr); return 1; }
  printf("OK %d keypoints, %d matches, levels %d, scale[7] %.7f\n", n, nm,
         extractor.GetLevels(), extractor.GetScaleFactors()[7]);
  return 0;
}
