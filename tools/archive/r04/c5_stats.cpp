// C5 resolve statistics on the CPU (diagnostic, not product): how often the
// sequential SearchByProjection(F, localMap) of the C5 problems
// (1920x1080, 4000 features, 50,000 synthetic map points, seed 5) needs more
// than the top-K candidates the GPU keeps per point (the "slow" re-scan of
// k_proj_resolve_fp), and how deep the claim dependencies inside a window of
// T points run (a lower bound on the fixed-point rounds per window).
// Build: g++ -O2 -std=c++17 -fopenmp -I include tools/r04/c5_stats.cpp -o /tmp/c5_stats
#include "../../oracle/orb_oracle.cpp"

#include <algorithm>
#include <cstdio>

int main(int argc, char** argv) {
  const int W = 1920, H = 1080, NF = 4000, M = 50000;
  const int P = argc > 1 ? atoi(argv[1]) : 4;
  const uint64_t seed = 5;
  float scale[8];
  scale[0] = 1.f;
  for (int l = 1; l < 8; ++l) scale[l] = scale[l - 1] * 1.2f;
  for (int p = 0; p < P; ++p) {
    std::vector<uint8_t> img((size_t)W * H);
    oracle_synth_image(seed, p, 0, W, H, img.data(), W);
    std::vector<orb_keypoint_t> kp(NF * 2);
    std::vector<uint8_t> desc(NF * 2 * 32);
    const int n = oracle_extract(img.data(), W, H, W, NF, 1.2f, 8, 20, 7, kp.data(), desc.data(),
                                 NF * 2, nullptr);
    std::vector<orb_mp_track_t> mps(M);
    std::vector<uint8_t> mpd((size_t)M * 32), lk(n);
    oracle_synth_local_map(seed + p, kp.data(), desc.data(), n, M, W, H, mps.data(), mpd.data(),
                           lk.data());
    Grid g;
    assign_grid(g, (const KP*)kp.data(), n, 0.f, (float)W, 0.f, (float)H);
    // candidate lists per point, sorted by distance (stable in scan order)
    std::vector<std::vector<std::pair<int, int>>> cand(M);
    std::vector<size_t> idxs;
    long long ncTot = 0, nIn = 0;
    int hist[6] = {0};
    for (int m = 0; m < M; ++m) {
      const orb_mp_track_t& mp = mps[m];
      if (!mp.in_view || mp.bad) continue;
      ++nIn;
      float r = (double)mp.view_cos > 0.998 ? 2.5f : 4.0f;
      const float rs = r * scale[mp.level];
      features_in_area(g, (const KP*)kp.data(), mp.proj_x, mp.proj_y, rs, mp.level - 1, mp.level,
                       idxs);
      for (size_t i : idxs) {
        if (lk[i]) continue;
        cand[m].push_back({descriptor_distance(mpd.data() + (size_t)m * 32, desc.data() + i * 32),
                           (int)i});
      }
      std::stable_sort(cand[m].begin(), cand[m].end(),
                       [](auto& a, auto& b) { return a.first < b.first; });
      ncTot += cand[m].size();
      hist[std::min<size_t>(5, cand[m].size())]++;
    }
    // sequential pass: slow points per K, claims
    const int Ks[3] = {4, 8, 16};
    int slow[3] = {0, 0, 0};
    std::vector<uint8_t> lock(lk.begin(), lk.end());
    std::vector<int> claimOf(M, -1), takenAt(n, -1);
    int matches = 0;
    for (int m = 0; m < M; ++m) {
      if (cand[m].empty()) continue;
      int found = 0;
      size_t j = 0;
      for (int kk = 0; kk < 3; ++kk) {
        int f = 0;
        for (size_t q = 0; q < cand[m].size() && q < (size_t)Ks[kk] && f < 2; ++q)
          if (!lock[cand[m][q].second]) ++f;
        if ((int)cand[m].size() > Ks[kk] && f < 2) ++slow[kk];
      }
      int bd = 256, bl = -1, bd2 = 256, bl2 = -1, bi = -1;
      for (j = 0; j < cand[m].size(); ++j) {
        const int i = cand[m][j].second, d = cand[m][j].first;
        if (lock[i]) continue;
        if (found == 0) { bd = d; bl = kp[i].octave; bi = i; }
        else if (found == 1) { bd2 = d; bl2 = kp[i].octave; }
        ++found;
        if (found == 2) break;
      }
      if (bd <= 100 && !(bl == bl2 && (float)bd > 0.8f * (float)bd2)) {
        ++matches;
        if (mps[m].has_obs) { lock[bi] = 1; claimOf[m] = bi; takenAt[bi] = m; }
      }
    }
    // dependency depth inside windows of T points: point m depends on the
    // earlier point of its window that took a keypoint among the candidates it
    // passed over or chose (up to its decision)
    for (int T : {256, 1024, 4096}) {
      long long sumDepth = 0;
      int nw = 0, maxD = 0;
      std::vector<int> depth(M, 0);
      for (int s = 0; s < M; s += T) {
        int wmax = 0;
        for (int m = s; m < std::min(M, s + T); ++m) {
          int d = 0;
          for (auto& c : cand[m]) {
            const int t = takenAt[c.second];
            if (t >= s && t < m) d = std::max(d, depth[t] + 1);
            if (t < 0 || t >= m) break;  // first free candidate reached: chosen (approx.)
          }
          depth[m] = d;
          wmax = std::max(wmax, d);
        }
        sumDepth += wmax;
        maxD = std::max(maxD, wmax);
        ++nw;
      }
      printf("  T=%d: windows %d, mean max-depth %.2f, worst %d\n", T, nw, (double)sumDepth / nw,
             maxD);
    }
    // the fixed-point (Jacobi) iteration itself over windows of T points:
    // rounds until no claim changes (k_proj_resolve_fp / k_proj_jacobi)
    for (int T : {1024, 4096, 16384, M}) {
      std::vector<int> lockC(lk.begin(), lk.end());  // committed: 1
      long long sumR = 0;
      int maxR = 0, nw = 0;
      for (int s0 = 0; s0 < M; s0 += T) {
        const int e0 = std::min(M, s0 + T);
        std::vector<int> claimPrev(n, INT32_MAX), claimCur(n, INT32_MAX), dec(e0 - s0, -2);
        int rounds = 0;
        while (true) {
          ++rounds;
          std::fill(claimCur.begin(), claimCur.end(), INT32_MAX);
          bool changed = false;
          for (int m = s0; m < e0; ++m) {
            int found = 0, bd = 256, bl = -1, bd2 = 256, bl2 = -1, bi = -1;
            for (auto& c : cand[m]) {
              const int i = c.second;
              if (lockC[i] || claimPrev[i] < m) continue;
              if (found == 0) { bd = c.first; bl = kp[i].octave; bi = i; }
              else { bd2 = c.first; bl2 = kp[i].octave; }
              if (++found == 2) break;
            }
            int acc = (bi >= 0 && bd <= 100 && !(bl == bl2 && (float)bd > 0.8f * (float)bd2)) ? bi : -1;
            const int claim = mps[m].has_obs ? acc : -1;
            if (claim >= 0) claimCur[claim] = std::min(claimCur[claim], m);
            if (dec[m - s0] != claim) changed = true;
            dec[m - s0] = claim;
          }
          std::swap(claimPrev, claimCur);
          if (!changed) break;
        }
        for (int m = s0; m < e0; ++m)
          if (dec[m - s0] >= 0) lockC[dec[m - s0]] = 1;
        sumR += rounds;
        maxR = std::max(maxR, rounds);
        ++nw;
      }
      printf("  Jacobi T=%d: windows %d, rounds mean %.2f max %d (total %lld)\n", T, nw,
             (double)sumR / nw, maxR, sumR);
    }
    printf("problem %d: n %d, in view %lld, mean cand %.2f, nc hist 0..5+ %d %d %d %d %d %d, "
           "slow K=4 %d K=8 %d K=16 %d, matches %d\n",
           p, n, nIn, (double)ncTot / nIn, hist[0], hist[1], hist[2], hist[3], hist[4], hist[5],
           slow[0], slow[1], slow[2], matches);
  }
  return 0;
}
