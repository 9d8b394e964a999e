// Probe: per-call cost of the host-buffer drop-in path through the C ABI
// (what ORBextractor::operator() / Frame::ComputeStereoMatches /
// ORBmatcher::SearchByProjection pay per frame), one call at a time as the
// reference's threads make them.  Also the per-stage kernel times of one
// single-image extraction (profiling mode, no graph).  PCIe-inclusive; quoted
// in INTEGRATION.md §4 and DESIGN.md §5, never the bench metric.
// Build: make -C tools/probe host_api_rate   Run: tools/probe/host_api_rate
#include <chrono>
#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <thread>
#include <vector>

#include "../../include/orb_abi.h"

static double now_ms() {
  return std::chrono::duration<double, std::milli>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define CHECK(x)                                                                   \
  do {                                                                             \
    orb_status_t s_ = (x);                                                         \
    if (s_ != ORB_OK) {                                                            \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, orb_status_string(s_)); \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

int main(int argc, char** argv) {
  const int W = 1241, H = 376, N = argc > 1 ? atoi(argv[1]) : 500;
  std::vector<std::vector<uint8_t>> imgs(16, std::vector<uint8_t>((size_t)W * H));
  for (int f = 0; f < 16; ++f) orb_synth_image(0x4B495454, f, 0, W, H, imgs[f].data(), W);
  orb_extractor_t* ext = nullptr;
  CHECK(orb_extractor_create(1000, 1.2f, 8, 20, 7, 0, &ext));
  const int cap = orb_extractor_capacity(ext, W, H);
  std::vector<orb_keypoint_t> kps(cap);
  std::vector<uint8_t> desc((size_t)cap * 32);
  int n = 0;
  for (int i = 0; i < 30; ++i)
    CHECK(orb_extractor_extract(ext, imgs[i % 16].data(), W, H, W, kps.data(), desc.data(), cap, &n));
  std::vector<double> t(N);
  for (int i = 0; i < N; ++i) {
    const double t0 = now_ms();
    CHECK(orb_extractor_extract(ext, imgs[i % 16].data(), W, H, W, kps.data(), desc.data(), cap, &n));
    t[i] = now_ms() - t0;
  }
  std::vector<double> s = t;
  std::sort(s.begin(), s.end());
  double sum = 0;
  for (double v : t) sum += v;
  printf("extract 1241x376 1000 feat (host buffers, 1 frame/call): median %.3f ms, mean %.3f ms, p90 %.3f ms -> %.0f frames/s\n",
         s[N / 2], sum / N, s[N * 9 / 10], 1e3 / (sum / N));
  // per-stage kernel time of one call (profiling mode launches without the graph)
  CHECK(orb_extractor_profile(ext, 1));
  for (int i = 0; i < 50; ++i)
    CHECK(orb_extractor_extract(ext, imgs[i % 16].data(), W, H, W, kps.data(), desc.data(), cap, &n));
  printf("  kernels per call (HIP events, 50 calls):");
  for (int st = 0; st <= 6; ++st) {
    double ms = 0;
    int launches = 0;
    const char* name = nullptr;
    CHECK(orb_extractor_profile_read(ext, st, &ms, &launches, &name));
    if (launches) printf(" %s %.3f ms;", name, ms / 50);
  }
  printf("\n");
  CHECK(orb_extractor_profile(ext, 0));

  // stereo: two 2000-feature extractors + ComputeStereoMatches on the handles
  orb_extractor_t *el = nullptr, *er = nullptr;
  CHECK(orb_extractor_create(2000, 1.2f, 8, 20, 7, 0, &el));
  CHECK(orb_extractor_create(2000, 1.2f, 8, 20, 7, 0, &er));
  orb_matcher_t* m = nullptr;
  CHECK(orb_matcher_create(0, &m));
  std::vector<uint8_t> il((size_t)W * H), ir((size_t)W * H);
  orb_synth_image(1, 0, 0, W, H, il.data(), W);
  orb_synth_image(1, 0, 1, W, H, ir.data(), W);
  const int cap2 = orb_extractor_capacity(el, W, H);
  std::vector<orb_keypoint_t> kl(cap2), kr(cap2);
  std::vector<uint8_t> dl((size_t)cap2 * 32), dr((size_t)cap2 * 32);
  std::vector<float> ur(cap2), dp(cap2);
  int nl = 0, nr = 0, nn = 0;
  const int NS = N / 2;
  double tx = 0, ts = 0;
  for (int i = 0; i < NS + 10; ++i) {
    const double t0 = now_ms();
    CHECK(orb_extractor_extract(el, il.data(), W, H, W, kl.data(), dl.data(), cap2, &nl));
    CHECK(orb_extractor_extract(er, ir.data(), W, H, W, kr.data(), dr.data(), cap2, &nr));
    const double t1 = now_ms();
    CHECK(orb_stereo_match_extracted(m, el, er, 386.1448f, 718.856f, ur.data(), dp.data(), cap2, &nn));
    const double t2 = now_ms();
    if (i >= 10) {
      tx += t1 - t0;
      ts += t2 - t1;
    }
  }
  printf("stereo pair 1241x376 2000+2000 feat: two extractions %.3f ms + ComputeStereoMatches on the handles %.3f ms per pair\n",
         tx / NS, ts / NS);
  // the same with the two extractions on two threads, as Frame's stereo
  // constructor runs them (src/Frame.cc:81-84): the handles' streams overlap
  double tc = 0;
  for (int i = 0; i < NS + 10; ++i) {
    const double t0 = now_ms();
    std::thread left([&] {
      CHECK(orb_extractor_extract(el, il.data(), W, H, W, kl.data(), dl.data(), cap2, &nl));
    });
    CHECK(orb_extractor_extract(er, ir.data(), W, H, W, kr.data(), dr.data(), cap2, &nr));
    left.join();
    CHECK(orb_stereo_match_extracted(m, el, er, 386.1448f, 718.856f, ur.data(), dp.data(), cap2, &nn));
    if (i >= 10) tc += now_ms() - t0;
  }
  printf("stereo pair, the two extractions on two threads: %.3f ms per pair incl. ComputeStereoMatches\n",
         tc / NS);

  // SearchByProjection(F, local map) on host buffers, 5000 map points
  std::vector<orb_mp_track_t> mps(5000);
  std::vector<uint8_t> mpd(5000 * 32), locked(n);
  orb_synth_local_map(1, kps.data(), desc.data(), n, 5000, W, H, mps.data(), mpd.data(), locked.data());
  float sf[8];
  orb_extractor_get_scale_factors(ext, sf);
  orb_frame_t fr{n, kps.data(), desc.data(), nullptr, 0.f, (float)W, 0.f, (float)H, 8, sf};
  std::vector<int32_t> km(n);
  int32_t nm = 0;
  for (int i = 0; i < 10; ++i)
    CHECK(orb_match_projection_local(m, &fr, locked.data(), 5000, mps.data(), mpd.data(), 1.f, 0.8f, km.data(), &nm));
  const double t0 = now_ms();
  for (int i = 0; i < N; ++i)
    CHECK(orb_match_projection_local(m, &fr, locked.data(), 5000, mps.data(), mpd.data(), 1.f, 0.8f, km.data(), &nm));
  printf("SearchByProjection (host buffers, %d kps, 5000 map points): %.3f ms per call (%d matches)\n",
         n, (now_ms() - t0) / N, nm);
  orb_matcher_destroy(m);
  orb_extractor_destroy(el);
  orb_extractor_destroy(er);
  orb_extractor_destroy(ext);
  return 0;
}
