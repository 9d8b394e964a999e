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

extern "C" int oracle_vocab_transform(int k, int L, int scoring, int weighting, int n_nodes,
                                      const int32_t* parent, const uint8_t* leaf,
                                      const uint8_t* node_desc, const double* node_weight, int n,
                                      const uint8_t* desc, int levelsup, uint32_t* bow_words,
                                      double* bow_values, int* n_words, uint32_t* fv_nodes,
                                      int32_t* fv_offs, uint32_t* fv_feats, int* n_fv,
                                      uint32_t* feat_word, uint32_t* feat_node);
extern "C" int oracle_match_bow(int n_kf, const uint8_t* kf_desc, const float* kf_angle,
                                const int32_t* kf_mp, const uint8_t* kf_mp_bad, int kf_nodes,
                                const uint32_t* kf_node_ids, const int32_t* kf_offs,
                                const uint32_t* kf_feats, int n_f, const uint8_t* f_desc,
                                const float* f_angle, int f_nodes, const uint32_t* f_node_ids,
                                const int32_t* f_offs, const uint32_t* f_feats, float nnratio,
                                int check_orientation, int32_t* f_match);

static uint64_t mix(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Frame::ComputeBoW (src/Frame.cc:439-449) through orb_amd::ORBVocabulary on a
// synthetic k=10, L=4 tree, then SearchByBoW(KF, F) on the resulting
// FeatureVectors; both checked against the oracle.
static int vocab_and_bow(const orb_amd::Descriptors& d1, const std::vector<orb_amd::KeyPoint>& k1,
                         const orb_amd::Descriptors& d2, const std::vector<orb_amd::KeyPoint>& k2) {
  const int k = 10, L = 4;
  std::vector<int32_t> parent(1, 0);
  std::vector<uint8_t> leaf(1, 0), nd(32, 0);
  std::vector<double> w(1, 0.0);
  uint64_t s = 99;
  std::vector<int> level(1, 0);
  for (size_t p = 0; p < parent.size(); ++p) {  // breadth-first: children of p
    if (level[p] == L) continue;
    for (int c = 0; c < k; ++c) {
      parent.push_back((int32_t)p);
      level.push_back(level[p] + 1);
      leaf.push_back(level[p] + 1 == L);
      for (int b = 0; b < 32; ++b) {
        const uint8_t flip = (uint8_t)(mix(s) & mix(s) & (level[p] > 1 ? mix(s) : 0xFF));
        nd.push_back((uint8_t)(nd[p * 32 + b] ^ flip));
      }
      w.push_back(level[p] + 1 == L ? 0.5 + (mix(s) % 1000) / 100.0 : 0.0);
    }
  }
  orb_amd::ORBVocabulary voc;
  voc.create(k, L, 0, 0, parent, leaf, nd, w);
  if (voc.size() != 10000 || voc.getBranchingFactor() != 10) {
    printf("FAIL vocabulary size %u\n", voc.size());
    return 1;
  }
  orb_amd::BowVector bow1, bow2;
  orb_amd::FeatureVector fv1, fv2;
  voc.transform(d1, bow1, fv1, 4);
  voc.transform(d2, bow2, fv2, 4);
  const int n = d1.rows;
  std::vector<uint32_t> bw(n), fvn(n), fvf(n), fw(n), fnode(n);
  std::vector<double> bv(n);
  std::vector<int32_t> fvo(n + 1);
  int nw = 0, nf = 0;
  oracle_vocab_transform(k, L, 0, 0, (int)parent.size(), parent.data(), leaf.data(), nd.data(),
                         w.data(), n, d1.data.data(), 4, bw.data(), bv.data(), &nw, fvn.data(),
                         fvo.data(), fvf.data(), &nf, fw.data(), fnode.data());
  if ((int)bow1.size() != nw || (int)fv1.size() != nf) {
    printf("FAIL transform sizes %zu/%d %zu/%d\n", bow1.size(), nw, fv1.size(), nf);
    return 1;
  }
  int i = 0;
  for (const auto& it : bow1) {
    if (it.first != bw[i] || memcmp(&it.second, &bv[i], 8)) { printf("FAIL BowVector\n"); return 1; }
    ++i;
  }
  i = 0;
  for (const auto& it : fv1) {
    if (it.first != fvn[i] ||
        it.second != std::vector<unsigned>(fvf.begin() + fvo[i], fvf.begin() + fvo[i + 1])) {
      printf("FAIL FeatureVector\n");
      return 1;
    }
    ++i;
  }
  orb_amd::FrameView KF, F;
  KF.mvKeysUn = k1; KF.mDescriptors = d1;
  F.mvKeysUn = k2; F.mDescriptors = d2;
  std::vector<int32_t> kfmp(KF.N()), out;
  std::vector<uint8_t> bad(KF.N(), 0);
  for (int j = 0; j < KF.N(); ++j) kfmp[j] = (mix(s) % 10) < 8 ? 1000 + j : -1;
  orb_amd::ORBmatcher m(0.75f, true);
  const int nm = m.SearchByBoW(KF, kfmp, bad, fv1, F, fv2, out);
  const orb_amd::CsrFeatureVector c1 = orb_amd::flatten(fv1), c2 = orb_amd::flatten(fv2);
  std::vector<float> a1(KF.N()), a2(F.N());
  for (int j = 0; j < KF.N(); ++j) a1[j] = k1[j].angle;
  for (int j = 0; j < F.N(); ++j) a2[j] = k2[j].angle;
  std::vector<int32_t> ref(F.N(), -1);
  const int nr = oracle_match_bow(KF.N(), d1.data.data(), a1.data(), kfmp.data(), bad.data(),
                                  c1.size(), c1.nodes.data(), c1.offs.data(), c1.feats.data(),
                                  F.N(), d2.data.data(), a2.data(), c2.size(), c2.nodes.data(),
                                  c2.offs.data(), c2.feats.data(), 0.75f, 1, ref.data());
  if (nm != nr || out != ref) { printf("FAIL SearchByBoW: gpu %d oracle %d\n", nm, nr); return 1; }
  fprintf(stderr, "bow: %zu words, %zu nodes, %d BoW matches\n", bow1.size(), fv1.size(), nm);
  return 0;
}

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
  {  // next frame of the sequence for the BoW chain
    std::vector<uint8_t> img2((size_t)W * H);
    orb_synth_image(77, 1, 0, W, H, img2.data(), W);
    std::vector<orb_amd::KeyPoint> kps2;
    orb_amd::Descriptors desc2;
    extractor({img2.data(), W, H, (size_t)W}, {}, kps2, desc2);
    if (vocab_and_bow(desc, kps, desc2, kps2)) return 1;
  }
  printf("OK %d keypoints, %d matches, levels %d, scale[7] %.7f\n", n, nm,
         extractor.GetLevels(), extractor.GetScaleFactors()[7]);
  return 0;
}
