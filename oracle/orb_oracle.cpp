// orb_oracle.cpp -- CPU ORACLE for the ORB hot path.  TEST INFRASTRUCTURE ONLY.
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
// load this library, and only as the checker / CPU baseline.  The product
// (lib/liborb_amd.so) never links or calls it.
//
// What it is: a scalar, single-threaded restatement of the reference's
// ORBextractor (src/ORBextractor.cc) and ORBmatcher / Frame matching code
// (src/ORBmatcher.cc, src/Frame.cc) of yg838457845/ORB_SLAM2-Chinese-annotation,
// with the OpenCV primitives it calls pinned to "OCV3-scalar" semantics
// (SURVEY.md Appendix A): FAST-9/16 + NMS, 8U INTER_LINEAR resize with 11-bit
// fixed-point weights, 8U 7x7 sigma-2 Gaussian with the integer kernel
// [18,34,49,55,49,34,18], OpenCV fastAtan2, round-half-even cvRound, and a
// pinned sin/cos (double evaluation, rounded to float).  Each function cites
// the reference lines it follows.  Control flow that the reference makes
// order-dependent (DistributeOctTree's std::list + pointer-sorted splits,
// the matchers' first-come claims) is restated literally with std::list and
// sequential loops; the pointer tie-break of src/ORBextractor.cc:703 is
// pinned to node creation order.
//
// PARITY STATUS: parity UNPINNED against a reference binary.  The reference
// cannot be built here (OpenCV/Eigen/Pangolin absent) and it
// ships no tests, fixtures or golden vectors.  What IS pinned:
// the constants the reference embeds (rBRIEF table, umax, per-level quotas,
// scale tables), checked against the reference source text by
// tests/test_oracle_constants.py when /root/reference is present, and the
// golden vectors under tests/golden/ generated from this file
// (tests/golden/make_golden.py) that freeze its behaviour.
//
// Build: oracle/Makefile (g++ -O2 -ffp-contract=off; no FMA contraction so the
// float expressions round exactly as written).

#include <limits.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <list>
#include <utility>
#include <vector>

#include "../include/orb_abi.h"
#include "../orb_slam2-chinese-annotation_amd/csrc/orb_pattern_data.h"
#include "../orb_slam2-chinese-annotation_amd/csrc/orb_synth.h"

namespace oracle {

typedef orb_keypoint_t KP;

// ---------------------------------------------------------------- A.5 rounding
static inline int cvRound(float v) { return (int)lrintf(v); }     // round half to even
static inline int cvRoundD(double v) { return (int)lrint(v); }
static inline int cvFloor(float v) { return (int)floorf(v); }
static inline int cvCeil(float v) { return (int)ceilf(v); }
static inline short sat_short(int v) { return (short)(v < -32768 ? -32768 : (v > 32767 ? 32767 : v)); }
static inline uint8_t sat_u8(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

struct Img {
  int w = 0, h = 0;
  std::vector<uint8_t> px;
  Img() {}
  Img(int w_, int h_) : w(w_), h(h_), px((size_t)w_ * h_) {}
  uint8_t at(int y, int x) const { return px[(size_t)y * w + x]; }
  uint8_t* row(int y) { return &px[(size_t)y * w]; }
  const uint8_t* row(int y) const { return &px[(size_t)y * w]; }
};

// ------------------------------------------------------------ a1: ctor tables
// src/ORBextractor.cc:428-489 (note `double scaleFactor`, include/ORBextractor.h:98)
struct Params {
  int nfeatures, nlevels, iniTh, minTh;
  double scaleFactor;
  std::vector<float> scale, invScale, sigma2, invSigma2;
  std::vector<int> quota;
  int umax[16];
};

static Params make_params(int nfeatures, float scaleFactorF, int nlevels, int iniTh, int minTh) {
  Params p;
  p.nfeatures = nfeatures;
  p.nlevels = nlevels;
  p.iniTh = iniTh;
  p.minTh = minTh;
  p.scaleFactor = (double)scaleFactorF;
  p.scale.assign(nlevels, 0.f);
  p.sigma2.assign(nlevels, 0.f);
  p.scale[0] = 1.0f;
  p.sigma2[0] = 1.0f;
  for (int i = 1; i < nlevels; ++i) {
    p.scale[i] = (float)((double)p.scale[i - 1] * p.scaleFactor);  // :439
    p.sigma2[i] = p.scale[i] * p.scale[i];                          // :440
  }
  p.invScale.resize(nlevels);
  p.invSigma2.resize(nlevels);
  for (int i = 0; i < nlevels; ++i) {
    p.invScale[i] = 1.0f / p.scale[i];
    p.invSigma2[i] = 1.0f / p.sigma2[i];
  }
  // :453-464 geometric per-level quotas
  p.quota.assign(nlevels, 0);
  const float factor = (float)(1.0f / p.scaleFactor);
  float nDesired = (float)nfeatures * (1 - factor) / (1 - (float)pow((double)factor, (double)nlevels));
  int sum = 0;
  for (int l = 0; l < nlevels - 1; ++l) {
    p.quota[l] = cvRound(nDesired);
    sum += p.quota[l];
    nDesired *= factor;
  }
  p.quota[nlevels - 1] = std::max(nfeatures - sum, 0);
  // :473-488 umax for the radius-15 circular patch
  const int HP = 15;
  int vmax = cvFloor(HP * sqrtf(2.f) / 2 + 1);
  int vmin = cvCeil(HP * sqrtf(2.f) / 2);
  const double hp2 = HP * HP;
  for (int v = 0; v <= vmax; ++v) p.umax[v] = cvRoundD(sqrt(hp2 - v * v));
  for (int v = HP, v0 = 0; v >= vmin; --v) {
    while (p.umax[v0] == p.umax[v0 + 1]) ++v0;
    p.umax[v] = v0;
    ++v0;
  }
  return p;
}

// ------------------------------------------------- a3: A.2 INTER_LINEAR resize
static Img resize_linear(const Img& src, int dw, int dh) {
  Img dst(dw, dh);
  const double scale_x = 1. / ((double)dw / src.w);
  const double scale_y = 1. / ((double)dh / src.h);
  std::vector<int> xofs(dw), yofs(dh);
  std::vector<short> ialpha(2 * dw), ibeta(2 * dh);
  int xmax = dw;
  for (int dx = 0; dx < dw; ++dx) {
    float fx = (float)((dx + 0.5) * scale_x - 0.5);
    int sx = cvFloor(fx);
    fx -= sx;
    if (sx < 0) { fx = 0; sx = 0; }
    if (sx + 1 >= src.w) {
      xmax = std::min(xmax, dx);
      if (sx >= src.w - 1) { fx = 0; sx = src.w - 1; }
    }
    xofs[dx] = sx;
    ialpha[2 * dx] = sat_short(cvRound((1.f - fx) * 2048));
    ialpha[2 * dx + 1] = sat_short(cvRound(fx * 2048));
  }
  for (int dy = 0; dy < dh; ++dy) {
    float fy = (float)((dy + 0.5) * scale_y - 0.5);
    int sy = cvFloor(fy);
    fy -= sy;
    yofs[dy] = sy;
    ibeta[2 * dy] = sat_short(cvRound((1.f - fy) * 2048));
    ibeta[2 * dy + 1] = sat_short(cvRound(fy * 2048));
  }
  std::vector<int> h0(dw), h1(dw);
  auto hpass = [&](int sy, std::vector<int>& D) {
    const uint8_t* S = src.row(sy);
    for (int dx = 0; dx < dw; ++dx) {
      const int sx = xofs[dx];
      D[dx] = dx < xmax ? S[sx] * ialpha[2 * dx] + S[sx + 1] * ialpha[2 * dx + 1] : S[sx] * 2048;
    }
  };
  for (int dy = 0; dy < dh; ++dy) {
    int s0 = yofs[dy], s1 = yofs[dy] + 1;
    s0 = s0 < 0 ? 0 : (s0 >= src.h ? src.h - 1 : s0);
    s1 = s1 < 0 ? 0 : (s1 >= src.h ? src.h - 1 : s1);
    hpass(s0, h0);
    hpass(s1, h1);
    const int b0 = ibeta[2 * dy], b1 = ibeta[2 * dy + 1];
    uint8_t* D = dst.row(dy);
    for (int dx = 0; dx < dw; ++dx) D[dx] = sat_u8((h0[dx] * b0 + h1[dx] * b1 + (1 << 21)) >> 22);
  }
  return dst;
}

// src/ORBextractor.cc:1172-1207 (the padding is never read by any consumer)
static std::vector<Img> compute_pyramid(const Params& p, const Img& image) {
  std::vector<Img> pyr(p.nlevels);
  pyr[0] = image;
  for (int l = 1; l < p.nlevels; ++l) {
    const float s = p.invScale[l];
    const int w = cvRound((float)image.w * s), h = cvRound((float)image.h * s);
    pyr[l] = resize_linear(pyr[l - 1], w, h);
  }
  return pyr;
}

// ----------------------------------------------------------- A.1 FAST-9/16
static const int kCircle[16][2] = {{0, 3},  {1, 3},   {2, 2},   {3, 1},   {3, 0},  {3, -1},
                                   {2, -2}, {1, -3},  {0, -3},  {-1, -3}, {-2, -2}, {-3, -1},
                                   {-3, 0}, {-3, 1},  {-2, 2},  {-1, 3}};

// OpenCV cornerScore<16>: max(t, best dark arc, best bright arc) - 1
static int corner_score(const int d[25], int threshold) {
  int a0 = threshold;
  for (int k = 0; k < 16; k += 2) {
    int a = std::min(d[k + 1], d[k + 2]);
    a = std::min(a, d[k + 3]);
    if (a <= a0) continue;
    for (int m = 4; m <= 8; ++m) a = std::min(a, d[k + m]);
    a0 = std::max(a0, std::min(a, d[k]));
    a0 = std::max(a0, std::min(a, d[k + 9]));
  }
  int b0 = -a0;
  for (int k = 0; k < 16; k += 2) {
    int b = std::max(d[k + 1], d[k + 2]);
    for (int m = 3; m <= 5; ++m) b = std::max(b, d[k + m]);
    if (b >= b0) continue;
    for (int m = 6; m <= 8; ++m) b = std::max(b, d[k + m]);
    b0 = std::min(b0, std::max(b, d[k]));
    b0 = std::min(b0, std::max(b, d[k + 9]));
  }
  return -b0 - 1;
}

// cv::FAST(roi, kps, threshold, nonmaxSuppression=true) on the ROI
// rows [y0,y1) x cols [x0,x1) of `img`; keypoints relative to the ROI.
static void fast_roi(const Img& img, int y0, int y1, int x0, int x1, int threshold,
                     std::vector<KP>& kps) {
  kps.clear();
  const int rows = y1 - y0, cols = x1 - x0;
  if (rows < 7 || cols < 7) return;
  threshold = std::min(std::max(threshold, 0), 255);
  std::vector<uint8_t> score((size_t)rows * cols, 0);
  std::vector<std::vector<int>> corners(rows);
  for (int i = 3; i < rows - 3; ++i) {
    for (int j = 3; j < cols - 3; ++j) {
      const int v = img.at(y0 + i, x0 + j);
      int ring[25];
      for (int k = 0; k < 16; ++k)
        ring[k] = img.at(y0 + i + kCircle[k][1], x0 + j + kCircle[k][0]);
      for (int k = 16; k < 25; ++k) ring[k] = ring[k - 16];
      // OpenCV FAST_t pre-tests on opposite circle pixels (necessary conditions
      // for a 9-arc; they only skip work, never change the result)
      auto cls = [&](int x) { return x < v - threshold ? 1 : (x > v + threshold ? 2 : 0); };
      int dm = cls(ring[0]) | cls(ring[8]);
      if (dm == 0) continue;
      dm &= cls(ring[2]) | cls(ring[10]);
      dm &= cls(ring[4]) | cls(ring[12]);
      dm &= cls(ring[6]) | cls(ring[14]);
      if (dm == 0) continue;
      dm &= cls(ring[1]) | cls(ring[9]);
      dm &= cls(ring[3]) | cls(ring[11]);
      dm &= cls(ring[5]) | cls(ring[13]);
      dm &= cls(ring[7]) | cls(ring[15]);
      if (dm == 0) continue;
      int d[25];
      for (int k = 0; k < 25; ++k) d[k] = v - ring[k];
      bool corner = false;
      int count = 0;
      for (int k = 0; k < 25 && !corner; ++k) {  // dark arc: x < v - t
        if (ring[k] < v - threshold) { if (++count > 8) corner = true; }
        else count = 0;
      }
      count = 0;
      for (int k = 0; k < 25 && !corner; ++k) {  // bright arc: x > v + t
        if (ring[k] > v + threshold) { if (++count > 8) corner = true; }
        else count = 0;
      }
      if (corner) {
        corners[i].push_back(j);
        score[(size_t)i * cols + j] = (uint8_t)corner_score(d, threshold);
      }
    }
  }
  for (int i = 3; i < rows - 3; ++i) {
    for (int j : corners[i]) {
      const int s = score[(size_t)i * cols + j];
      bool keep = true;
      for (int dy = -1; dy <= 1 && keep; ++dy)
        for (int dx = -1; dx <= 1; ++dx) {
          if (!dy && !dx) continue;
          if (!(s > score[(size_t)(i + dy) * cols + j + dx])) { keep = false; break; }
        }
      if (keep) {
        KP k;
        k.x = (float)j;
        k.y = (float)i;
        k.size = 7.f;
        k.angle = -1.f;
        k.response = (float)s;
        k.octave = 0;
        k.class_id = -1;
        kps.push_back(k);
      }
    }
  }
}

// ------------------------------------------------ a5: DistributeOctTree
// src/ORBextractor.cc:500-556 (DivideNode), :558-782 (DistributeOctTree)
struct Node {
  std::vector<KP> keys;
  int ulx, uly, urx, ury, blx, bly, brx, bry;
  std::list<Node>::iterator lit;
  bool noMore = false;
  long seq = 0;  // creation order: stands in for the node's heap address (H2)
};

static void divide_node(const Node& p, Node& n1, Node& n2, Node& n3, Node& n4) {
  const int halfX = (int)ceilf((float)(p.urx - p.ulx) / 2);
  const int halfY = (int)ceilf((float)(p.bry - p.uly) / 2);
  n1.ulx = p.ulx; n1.uly = p.uly;
  n1.urx = p.ulx + halfX; n1.ury = p.uly;
  n1.blx = p.ulx; n1.bly = p.uly + halfY;
  n1.brx = p.ulx + halfX; n1.bry = p.uly + halfY;
  n2.ulx = n1.urx; n2.uly = n1.ury;
  n2.urx = p.urx; n2.ury = p.ury;
  n2.blx = n1.brx; n2.bly = n1.bry;
  n2.brx = p.urx; n2.bry = p.uly + halfY;
  n3.ulx = n1.blx; n3.uly = n1.bly;
  n3.urx = n1.brx; n3.ury = n1.bry;
  n3.blx = p.blx; n3.bly = p.bly;
  n3.brx = n1.brx; n3.bry = p.bly;
  n4.ulx = n3.urx; n4.uly = n3.ury;
  n4.urx = n2.brx; n4.ury = n2.bry;
  n4.blx = n3.brx; n4.bly = n3.bry;
  n4.brx = p.brx; n4.bry = p.bry;
  for (const KP& k : p.keys) {
    if (k.x < n1.urx) {
      if (k.y < n1.bry) n1.keys.push_back(k);
      else n3.keys.push_back(k);
    } else if (k.y < n1.bry) {
      n2.keys.push_back(k);
    } else {
      n4.keys.push_back(k);
    }
  }
  if (n1.keys.size() == 1) n1.noMore = true;
  if (n2.keys.size() == 1) n2.noMore = true;
  if (n3.keys.size() == 1) n3.noMore = true;
  if (n4.keys.size() == 1) n4.noMore = true;
}

static std::vector<KP> distribute_oct_tree(const std::vector<KP>& toDistribute, int minX, int maxX,
                                           int minY, int maxY, int N) {
  const int nIni = (int)roundf((float)(maxX - minX) / (maxY - minY));
  const float hX = (float)(maxX - minX) / nIni;
  std::list<Node> nodes;
  long seq = 0;
  std::vector<Node*> ini(nIni);
  for (int i = 0; i < nIni; ++i) {
    Node n;
    n.ulx = (int)(hX * (float)i); n.uly = 0;
    n.urx = (int)(hX * (float)(i + 1)); n.ury = 0;
    n.blx = n.ulx; n.bly = maxY - minY;
    n.brx = n.urx; n.bry = maxY - minY;
    n.seq = seq++;
    nodes.push_back(n);
    ini[i] = &nodes.back();
  }
  for (const KP& k : toDistribute) ini[(size_t)(k.x / hX)]->keys.push_back(k);
  for (auto it = nodes.begin(); it != nodes.end();) {
    if (it->keys.size() == 1) { it->noMore = true; ++it; }
    else if (it->keys.empty()) it = nodes.erase(it);
    else ++it;
  }

  typedef std::pair<int, Node*> SP;
  auto sp_less = [](const SP& a, const SP& b) {
    if (a.first != b.first) return a.first < b.first;
    return a.second->seq < b.second->seq;  // pinned pointer order (H2)
  };
  std::vector<SP> sizeAndNode;
  bool finish = false;
  auto add_child = [&](Node& c, bool countExpand, int& nToExpand) {
    if (c.keys.empty()) return;
    c.seq = seq++;
    nodes.push_front(c);
    if (c.keys.size() > 1) {
      if (countExpand) ++nToExpand;
      sizeAndNode.push_back(SP((int)c.keys.size(), &nodes.front()));
      nodes.front().lit = nodes.begin();
    }
  };
  while (!finish) {
    const int prevSize = (int)nodes.size();
    int nToExpand = 0;
    sizeAndNode.clear();
    for (auto it = nodes.begin(); it != nodes.end();) {
      if (it->noMore) { ++it; continue; }
      Node n1, n2, n3, n4;
      divide_node(*it, n1, n2, n3, n4);
      add_child(n1, true, nToExpand);
      add_child(n2, true, nToExpand);
      add_child(n3, true, nToExpand);
      add_child(n4, true, nToExpand);
      it = nodes.erase(it);
    }
    if ((int)nodes.size() >= N || (int)nodes.size() == prevSize) {
      finish = true;
    } else if ((int)nodes.size() + nToExpand * 3 > N) {
      while (!finish) {
        const int prev = (int)nodes.size();
        std::vector<SP> prevSizeAndNode = sizeAndNode;
        sizeAndNode.clear();
        std::sort(prevSizeAndNode.begin(), prevSizeAndNode.end(), sp_less);
        int dummy = 0;
        for (int j = (int)prevSizeAndNode.size() - 1; j >= 0; --j) {
          Node n1, n2, n3, n4;
          Node* parent = prevSizeAndNode[j].second;
          divide_node(*parent, n1, n2, n3, n4);
          add_child(n1, false, dummy);
          add_child(n2, false, dummy);
          add_child(n3, false, dummy);
          add_child(n4, false, dummy);
          nodes.erase(parent->lit);
          if ((int)nodes.size() >= N) break;
        }
        if ((int)nodes.size() >= N || (int)nodes.size() == prev) finish = true;
      }
    }
  }
  std::vector<KP> result;
  result.reserve(nodes.size());
  for (const Node& n : nodes) {  // :763-779 first max response in node order
    const KP* best = &n.keys[0];
    float maxResp = best->response;
    for (size_t k = 1; k < n.keys.size(); ++k)
      if (n.keys[k].response > maxResp) { best = &n.keys[k]; maxResp = n.keys[k].response; }
    result.push_back(*best);
  }
  return result;
}

// --------------------------------------------------------- a4: cells + octree
// src/ORBextractor.cc:785-892
struct LevelCandidates {
  std::vector<KP> keys;  // vToDistributeKeys (relative to the border origin)
};

static void level_candidates(const Params& p, const Img& lvl, std::vector<KP>& toDistribute) {
  const float W = 30;
  const int minBorderX = 19 - 3, minBorderY = minBorderX;
  const int maxBorderX = lvl.w - 19 + 3, maxBorderY = lvl.h - 19 + 3;
  toDistribute.clear();
  const float width = (float)(maxBorderX - minBorderX);
  const float height = (float)(maxBorderY - minBorderY);
  const int nCols = (int)(width / W), nRows = (int)(height / W);
  const int wCell = (int)ceilf(width / nCols), hCell = (int)ceilf(height / nRows);
  std::vector<KP> cell;
  for (int i = 0; i < nRows; ++i) {
    const float iniY = (float)(minBorderY + i * hCell);
    float maxY = iniY + hCell + 6;
    if (iniY >= maxBorderY - 3) continue;
    if (maxY > maxBorderY) maxY = (float)maxBorderY;
    for (int j = 0; j < nCols; ++j) {
      const float iniX = (float)(minBorderX + j * wCell);
      float maxX = iniX + wCell + 6;
      if (iniX >= maxBorderX - 6) continue;
      if (maxX > maxBorderX) maxX = (float)maxBorderX;
      fast_roi(lvl, (int)iniY, (int)maxY, (int)iniX, (int)maxX, p.iniTh, cell);
      if (cell.empty()) fast_roi(lvl, (int)iniY, (int)maxY, (int)iniX, (int)maxX, p.minTh, cell);
      for (KP k : cell) {
        k.x += j * wCell;
        k.y += i * hCell;
        toDistribute.push_back(k);
      }
    }
  }
}

// a6: IC_Angle + A.4 fastAtan2, src/ORBextractor.cc:77-113
static float fast_atan2(float y, float x) {
  const float r2d = (float)(180 / M_PI);
  const float p1 = 0.9997878412794807f * r2d, p3 = -0.3258083974640975f * r2d;
  const float p5 = 0.1555786518463281f * r2d, p7 = -0.04432655554792128f * r2d;
  const float ax = fabsf(x), ay = fabsf(y);
  float a, c, c2;
  if (ax >= ay) {
    c = ay / (ax + (float)2.2204460492503131e-16);
    c2 = c * c;
    a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  } else {
    c = ax / (ay + (float)2.2204460492503131e-16);
    c2 = c * c;
    a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  }
  if (x < 0) a = 180.f - a;
  if (y < 0) a = 360.f - a;
  return a;
}

static float ic_angle(const Img& img, float px, float py, const int* umax) {
  int m01 = 0, m10 = 0;
  const int cy = cvRound(py), cx = cvRound(px);
  for (int u = -15; u <= 15; ++u) m10 += u * img.at(cy, cx + u);
  for (int v = 1; v <= 15; ++v) {
    int vsum = 0;
    const int d = umax[v];
    for (int u = -d; u <= d; ++u) {
      const int plus = img.at(cy + v, cx + u), minus = img.at(cy - v, cx + u);
      vsum += plus - minus;
      m10 += u * (plus + minus);
    }
    m01 += v * vsum;
  }
  return fast_atan2((float)m01, (float)m10);
}

// a7: A.3 GaussianBlur 7x7 sigma 2, BORDER_REFLECT_101, src/ORBextractor.cc:1143-1145
static inline int reflect101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) {
    if (i < 0) i = -i;
    if (i >= n) i = 2 * n - 2 - i;
  }
  return i;
}

static Img gaussian_blur7(const Img& src) {
  static const int k[7] = {18, 34, 49, 55, 49, 34, 18};
  Img dst(src.w, src.h);
  std::vector<int> rowsum((size_t)src.w * src.h);
  for (int y = 0; y < src.h; ++y)
    for (int x = 0; x < src.w; ++x) {
      int s = 0;
      for (int i = 0; i < 7; ++i) s += k[i] * src.at(y, reflect101(x + i - 3, src.w));
      rowsum[(size_t)y * src.w + x] = s;
    }
  for (int y = 0; y < src.h; ++y)
    for (int x = 0; x < src.w; ++x) {
      int s = 0;
      for (int j = 0; j < 7; ++j) s += k[j] * rowsum[(size_t)reflect101(y + j - 3, src.h) * src.w + x];
      dst.row(y)[x] = sat_u8((s + (1 << 15)) >> 16);
    }
  return dst;
}

// A.6 pinned sin/cos: fdlibm-style reduction and kernels in double, rounded to float.
[[maybe_unused]] static void pinned_sincos(float angle, float* s_out, float* c_out) {
  const double x = (double)angle;
  const double invpio2 = 6.36619772367581382433e-01;
  const double pio2_1 = 1.57079632673412561417e+00, pio2_1t = 6.07710050650619224932e-11;
  const double k = nearbyint(x * invpio2);
  const double r = (x - k * pio2_1) - k * pio2_1t;
  const double z = r * r;
  const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
               S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
               S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
  const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
               C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
               C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
  const double ps = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
  const double sn = r + (z * r) * (S1 + z * ps);
  const double pc = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
  const double hz = 0.5 * z, w = 1.0 - hz;
  const double cs = w + (((1.0 - w) - hz) + z * pc);
  const int q = ((int)k) & 3;
  double s, c;
  switch (q) {
    case 0: s = sn; c = cs; break;
    case 1: s = cs; c = -sn; break;
    case 2: s = -sn; c = -cs; break;
    default: s = -cs; c = sn; break;
  }
  *s_out = (float)s;
  *c_out = (float)c;
}

// ORB_ORACLE_GLIBC_MATH (oracle/Makefile target liborb_oracle_glibc.so; used
// only by tools/parity_libm.py to measure what the A.6/A.7 pins change): the
// reference's own calls instead of the pins -- cos/sin of a float under
// `using namespace std` (src/ORBextractor.cc:67-68,125), i.e. glibc cosf/sinf.
static inline void desc_sincos(float angle, float* s, float* c) {
#ifdef ORB_ORACLE_GLIBC_MATH
  *s = std::sin(angle);
  *c = std::cos(angle);
#else
  pinned_sincos(angle, s, c);
#endif
}

// a8: computeOrbDescriptor, src/ORBextractor.cc:119-164
static void orb_descriptor(const KP& kpt, const Img& blurred, uint8_t* desc) {
  const float factorPI = (float)(M_PI / 180.f);
  const float angle = kpt.angle * factorPI;
  float a, b;
  {
    float s, c;
    desc_sincos(angle, &s, &c);
    a = c;
    b = s;
  }
  const int cy = cvRound(kpt.y), cx = cvRound(kpt.x);
  auto value = [&](int idx) -> int {
    const float px = (float)kOrbPatternXY[2 * idx], py = (float)kOrbPatternXY[2 * idx + 1];
    const int dy = cvRound(px * b + py * a);
    const int dx = cvRound(px * a - py * b);
    return blurred.at(cy + dy, cx + dx);
  };
  for (int i = 0; i < 32; ++i) {
    int val = 0;
    for (int bit = 0; bit < 8; ++bit) {
      const int t0 = value(16 * i + 2 * bit), t1 = value(16 * i + 2 * bit + 1);
      val |= (t0 < t1) << bit;
    }
    desc[i] = (uint8_t)val;
  }
}

// a2: operator(), src/ORBextractor.cc:1091-1169
struct ExtractResult {
  std::vector<KP> keys;
  std::vector<uint8_t> desc;
  std::vector<Img> pyramid;
  std::vector<std::vector<KP>> candidates;  // per level, vToDistributeKeys
  std::vector<int> perLevel;
};

static void extract(const Params& p, const Img& image, ExtractResult& out) {
  out.pyramid = compute_pyramid(p, image);
  std::vector<std::vector<KP>> all(p.nlevels);
  out.candidates.assign(p.nlevels, {});
  for (int l = 0; l < p.nlevels; ++l) {
    const Img& lvl = out.pyramid[l];
    std::vector<KP>& cand = out.candidates[l];
    level_candidates(p, lvl, cand);
    const int minBorderX = 16, minBorderY = 16;
    const int maxBorderX = lvl.w - 16, maxBorderY = lvl.h - 16;
    all[l] = distribute_oct_tree(cand, minBorderX, maxBorderX, minBorderY, maxBorderY, p.quota[l]);
    const int scaledPatchSize = (int)(31 * p.scale[l]);
    for (KP& k : all[l]) {
      k.x += minBorderX;
      k.y += minBorderY;
      k.octave = l;
      k.size = (float)scaledPatchSize;
    }
  }
  for (int l = 0; l < p.nlevels; ++l)
    for (KP& k : all[l]) k.angle = ic_angle(out.pyramid[l], k.x, k.y, p.umax);
  int total = 0;
  out.perLevel.assign(p.nlevels, 0);
  for (int l = 0; l < p.nlevels; ++l) total += out.perLevel[l] = (int)all[l].size();
  out.keys.clear();
  out.keys.reserve(total);
  out.desc.assign((size_t)total * 32, 0);
  int offset = 0;
  for (int l = 0; l < p.nlevels; ++l) {
    if (all[l].empty()) continue;
    const Img blurred = gaussian_blur7(out.pyramid[l]);
    for (size_t i = 0; i < all[l].size(); ++i)
      orb_descriptor(all[l][i], blurred, &out.desc[(size_t)(offset + i) * 32]);
    offset += (int)all[l].size();
    if (l != 0) {
      const float scale = p.scale[l];
      for (KP& k : all[l]) { k.x *= scale; k.y *= scale; }
    }
    out.keys.insert(out.keys.end(), all[l].begin(), all[l].end());
  }
}

// ----------------------------------------------------------------- matcher
// a10: DescriptorDistance, src/ORBmatcher.cc:1814-1830
static int descriptor_distance(const uint8_t* a, const uint8_t* b) {
  int dist = 0;
  for (int i = 0; i < 8; ++i) {
    uint32_t pa, pb;
    memcpy(&pa, a + 4 * i, 4);
    memcpy(&pb, b + 4 * i, 4);
    uint32_t v = pa ^ pb;
    v = v - ((v >> 1) & 0x55555555);
    v = (v & 0x33333333) + ((v >> 2) & 0x33333333);
    dist += (((v + (v >> 4)) & 0xF0F0F0F) * 0x1010101) >> 24;
  }
  return dist;
}

// a12 + a13: Frame grid, src/Frame.cc:261-276, 368-436
struct Grid {
  float minX, maxX, minY, maxY, invW, invH;
  std::vector<size_t> cell[ORB_GRID_COLS][ORB_GRID_ROWS];
};

static void assign_grid(Grid& g, const KP* keys, int n, float minX, float maxX, float minY,
                        float maxY) {
  g.minX = minX; g.maxX = maxX; g.minY = minY; g.maxY = maxY;
  g.invW = (float)ORB_GRID_COLS / (maxX - minX);
  g.invH = (float)ORB_GRID_ROWS / (maxY - minY);
  for (int i = 0; i < ORB_GRID_COLS; ++i)
    for (int j = 0; j < ORB_GRID_ROWS; ++j) g.cell[i][j].clear();
  for (int i = 0; i < n; ++i) {
    const int px = (int)roundf((keys[i].x - minX) * g.invW);
    const int py = (int)roundf((keys[i].y - minY) * g.invH);
    if (px < 0 || px >= ORB_GRID_COLS || py < 0 || py >= ORB_GRID_ROWS) continue;
    g.cell[px][py].push_back((size_t)i);
  }
}

static void features_in_area(const Grid& g, const KP* keys, float x, float y, float r,
                             int minLevel, int maxLevel, std::vector<size_t>& out) {
  out.clear();
  const int nMinCellX = std::max(0, (int)floorf((x - g.minX - r) * g.invW));
  if (nMinCellX >= ORB_GRID_COLS) return;
  const int nMaxCellX = std::min(ORB_GRID_COLS - 1, (int)ceilf((x - g.minX + r) * g.invW));
  if (nMaxCellX < 0) return;
  const int nMinCellY = std::max(0, (int)floorf((y - g.minY - r) * g.invH));
  if (nMinCellY >= ORB_GRID_ROWS) return;
  const int nMaxCellY = std::min(ORB_GRID_ROWS - 1, (int)ceilf((y - g.minY + r) * g.invH));
  if (nMaxCellY < 0) return;
  const bool checkLevels = (minLevel > 0) || (maxLevel >= 0);
  for (int ix = nMinCellX; ix <= nMaxCellX; ++ix)
    for (int iy = nMinCellY; iy <= nMaxCellY; ++iy)
      for (size_t idx : g.cell[ix][iy]) {
        const KP& k = keys[idx];
        if (checkLevels) {
          if (k.octave < minLevel) continue;
          if (maxLevel >= 0 && k.octave > maxLevel) continue;
        }
        const float dx = k.x - x, dy = k.y - y;
        if (fabsf(dx) < r && fabsf(dy) < r) out.push_back(idx);
      }
}

// a15: SearchByProjection(Frame&, const vector<MapPoint*>&, float th), src/ORBmatcher.cc:47-141
static int search_by_projection_local(const orb_frame_t* F, const uint8_t* kp_locked, int nmp,
                                      const orb_mp_track_t* mps, const uint8_t* mp_desc,
                                      float th, float nnratio, int32_t* kp_match) {
  thread_local Grid g;  // per thread: the oracle runs on many host threads (bench.py cpu_all_cores)
  assign_grid(g, F->keys, F->n, F->min_x, F->max_x, F->min_y, F->max_y);
  // lock[i]: F.mvpMapPoints[i] && ->Observations() > 0 ; updated by claims of has_obs points
  std::vector<uint8_t> lock(F->n);
  for (int i = 0; i < F->n; ++i) {
    lock[i] = kp_locked ? kp_locked[i] : 0;
    kp_match[i] = -1;
  }
  const bool bFactor = th != 1.0f;
  int nmatches = 0;
  std::vector<size_t> idxs;
  for (int m = 0; m < nmp; ++m) {
    const orb_mp_track_t& mp = mps[m];
    if (!mp.in_view || mp.bad) continue;
    const int lvl = mp.level;
    float r = (double)mp.view_cos > 0.998 ? 2.5f : 4.0f;  // float vs double literal (:137)
    if (bFactor) r *= th;
    const float rs = r * F->scale_factors[lvl];
    features_in_area(g, F->keys, mp.proj_x, mp.proj_y, rs, lvl - 1, lvl, idxs);
    if (idxs.empty()) continue;
    const uint8_t* d = mp_desc + (size_t)m * 32;
    int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
    for (size_t idx : idxs) {
      if (lock[idx]) continue;
      if (F->u_right && F->u_right[idx] > 0) {
        const float er = fabsf(mp.proj_xr - F->u_right[idx]);
        if (er > r * F->scale_factors[lvl]) continue;
      }
      const int dist = descriptor_distance(d, F->descriptors + idx * 32);
      if (dist < bestDist) {
        bestDist2 = bestDist;
        bestDist = dist;
        bestLevel2 = bestLevel;
        bestLevel = F->keys[idx].octave;
        bestIdx = (int)idx;
      } else if (dist < bestDist2) {
        bestLevel2 = F->keys[idx].octave;
        bestDist2 = dist;
      }
    }
    if (bestDist <= 100) {
      if (bestLevel == bestLevel2 && (float)bestDist > nnratio * (float)bestDist2) continue;
      kp_match[bestIdx] = m;
      if (mp.has_obs) lock[bestIdx] = 1;
      ++nmatches;
    }
  }
  return nmatches;
}

// a18: ComputeThreeMaxima, src/ORBmatcher.cc:1765-1809
// ---------------------------------------------------------------- frustum
// A.7 pinned log: the fdlibm e_log scheme in double (x = 2^k (1+f),
// s = f/(2+f), R = degree-14 polynomial in s^2).  MapPoint::PredictScale's
// log(float) is pinned to (float)pinned_log((double)ratio).
static double pinned_log(double x) {
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  const double L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01,
               L3 = 2.857142874366239149e-01, L4 = 2.222219843214978396e-01,
               L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01,
               L7 = 1.479819860511658591e-01;
  if (!(x > 0.0)) return x == 0.0 ? -INFINITY : NAN;
  if (isinf(x)) return x;
  uint64_t bits;
  memcpy(&bits, &x, 8);
  int32_t hi = (int32_t)(bits >> 32);
  const uint32_t lo = (uint32_t)bits;
  int k = (hi >> 20) - 1023;
  hi &= 0x000fffff;
  const int32_t up = (hi + 0x95f64) & 0x100000;  // mantissa >= sqrt(2): halve it
  const uint64_t mb = ((uint64_t)(uint32_t)(hi | (up ^ 0x3ff00000)) << 32) | lo;
  double mant;
  memcpy(&mant, &mb, 8);
  k += up >> 20;
  const double f = mant - 1.0, dk = (double)k;
  if ((0x000fffff & (2 + hi)) < 3) {
    if (f == 0.0) return k == 0 ? 0.0 : dk * ln2_hi + dk * ln2_lo;
    const double R = f * f * (0.5 - 0.33333333333333333 * f);
    return k == 0 ? f - R : dk * ln2_hi - ((R - dk * ln2_lo) - f);
  }
  const double sv = f / (2.0 + f), z = sv * sv, w = z * z;
  const double R = z * (L1 + w * (L3 + w * (L5 + w * L7))) + w * (L2 + w * (L4 + w * L6));
  if (((hi - 0x6147a) | (0x6b851 - hi)) > 0) {
    const double hf = 0.5 * f * f;
    return k == 0 ? f - (hf - sv * (hf + R))
                  : dk * ln2_hi - ((hf - (sv * (hf + R) + dk * ln2_lo)) - f);
  }
  return k == 0 ? f - sv * (f - R) : dk * ln2_hi - ((sv * (f - R) - dk * ln2_lo) - f);
}

// log(ratio) of MapPoint::PredictScale (src/MapPoint.cc:443): pinned, or glibc
// logf under ORB_ORACLE_GLIBC_MATH (see desc_sincos)
static inline float scale_log(float ratio) {
#ifdef ORB_ORACLE_GLIBC_MATH
  return std::log(ratio);
#else
  return (float)pinned_log((double)ratio);
#endif
}

struct FrustumCfg {
  orb_camera_t cam;
  float minX, maxX, minY, maxY, cosLimit, logScale;
  int nLevels;
};

// Frame::isInFrustum (src/Frame.cc:303-366) for one MapPoint; true = in view.
// Pinned arithmetic: Pc = Rcw*P + tcw as float dot products left to right
// then + t (cv::gemm's 3x3 float path); cv::norm(PO) = sqrt of a double sum
// of squares (normL2Sqr<float,double>), returned as double and stored as float
// (:339); PO.dot(Pn) accumulates in double (dotProd_32f), divided in double by
// the float dist (:351); PredictScale (src/MapPoint.cc:435-450) in float with
// logf pinned above.
static bool frustum_one(const orb_map_point_t& mp, const orb_pose_t& T, const FrustumCfg& c,
                        orb_mp_track_t& tr) {
  const float P0 = mp.pos[0], P1 = mp.pos[1], P2 = mp.pos[2];
  const float X = ((T.rcw[0] * P0 + T.rcw[1] * P1) + T.rcw[2] * P2) + T.tcw[0];
  const float Y = ((T.rcw[3] * P0 + T.rcw[4] * P1) + T.rcw[5] * P2) + T.tcw[1];
  const float Z = ((T.rcw[6] * P0 + T.rcw[7] * P1) + T.rcw[8] * P2) + T.tcw[2];
  if (Z < 0.0f) return false;                                   // :320-321
  const float invz = 1.0f / Z;                                  // :325
  const float u = c.cam.fx * X * invz + c.cam.cx;
  const float v = c.cam.fy * Y * invz + c.cam.cy;
  if (u < c.minX || u > c.maxX) return false;                   // :329-332
  if (v < c.minY || v > c.maxY) return false;
  const float maxDistance = 1.2f * mp.max_distance;             // src/MapPoint.cc:410-414
  const float minDistance = 0.8f * mp.min_distance;             // src/MapPoint.cc:404-408
  const float O0 = P0 - T.ow[0], O1 = P1 - T.ow[1], O2 = P2 - T.ow[2];
  double ss = 0.0;
  ss += (double)O0 * O0;
  ss += (double)O1 * O1;
  ss += (double)O2 * O2;
  const float dist = (float)sqrt(ss);                           // :339
  if (dist < minDistance || dist > maxDistance) return false;   // :341-342
  double dot = 0.0;
  dot += (double)O0 * mp.normal[0];
  dot += (double)O1 * mp.normal[1];
  dot += (double)O2 * mp.normal[2];
  const float viewCos = (float)(dot / (double)dist);            // :351
  if (viewCos < c.cosLimit) return false;                       // :353-354
  const float ratio = mp.max_distance / dist;                   // PredictScale
  const float lr = scale_log(ratio);
  const float q = ceilf(lr / c.logScale);
  int level;
  if (q < 0.f) level = 0;
  else if (q >= (float)c.nLevels) level = c.nLevels - 1;
  else level = (int)q;
  tr.proj_x = u;                                                // :362-368
  tr.proj_xr = u - c.cam.bf * invz;
  tr.proj_y = v;
  tr.level = level;
  tr.view_cos = viewCos;
  return true;
}

// Tracking::SearchLocalPoints' frustum loop (src/Tracking.cc:1360-1377).
static int frustum_all(int n, const orb_map_point_t* mps, const orb_pose_t& T,
                       const FrustumCfg& c, orb_mp_track_t* tracks) {
  int nToMatch = 0;
  for (int i = 0; i < n; ++i) {
    orb_mp_track_t tr;
    memset(&tr, 0, sizeof(tr));
    tr.bad = mps[i].bad;
    tr.has_obs = mps[i].has_obs;
    if (!mps[i].seen && !mps[i].bad && frustum_one(mps[i], T, c, tr)) {
      tr.in_view = 1;
      ++nToMatch;
    }
    tracks[i] = tr;
  }
  return nToMatch;
}

static void three_maxima(const std::vector<int>* histo, int L, int& ind1, int& ind2, int& ind3) {
  int max1 = 0, max2 = 0, max3 = 0;
  for (int i = 0; i < L; ++i) {
    const int s = (int)histo[i].size();
    if (s > max1) {
      max3 = max2; max2 = max1; max1 = s;
      ind3 = ind2; ind2 = ind1; ind1 = i;
    } else if (s > max2) {
      max3 = max2; max2 = s;
      ind3 = ind2; ind2 = i;
    } else if (s > max3) {
      max3 = s; ind3 = i;
    }
  }
  if (max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
  else if (max3 < 0.1f * (float)max1) { ind3 = -1; }
}

static inline int rot_bin(float rot) {  // src/ORBmatcher.cc:1582-1588 (factor bug kept)
  const float factor = 1.0f / 30;
  if (rot < 0.0) rot += 360.0f;
  int bin = (int)roundf(rot * factor);
  if (bin == 30) bin = 0;
  return bin;
}

// a16: SearchByProjection(Frame&, const Frame&, float, bool), src/ORBmatcher.cc:1460-1619
static int search_by_projection_frame(const orb_frame_t* C, const uint8_t* kp_locked, int nlast,
                                      const orb_last_mp_t* last, const uint8_t* last_desc,
                                      const orb_camera_t* cam, float tlc_z, float th, int mono,
                                      int checkOri, int32_t* kp_match) {
  thread_local Grid g;  // per thread: the oracle runs on many host threads (bench.py cpu_all_cores)
  assign_grid(g, C->keys, C->n, C->min_x, C->max_x, C->min_y, C->max_y);
  // state[i]: 0 untouched, 1 assigned this call (holder slot[i]), 2 cleared this call
  std::vector<int> slot(C->n, -1), state(C->n, 0);
  std::vector<uint8_t> locked(C->n, 0);  // mvpMapPoints[i] && Observations() > 0
  for (int i = 0; i < C->n; ++i) locked[i] = kp_locked ? kp_locked[i] : 0;
  std::vector<int> rotHist[30];
  const bool bForward = tlc_z > cam->mb && !mono;
  const bool bBackward = -tlc_z > cam->mb && !mono;
  int nmatches = 0;
  std::vector<size_t> idxs;
  for (int i = 0; i < nlast; ++i) {
    const orb_last_mp_t& L = last[i];
    if (!L.valid) continue;
    const float invzc = L.invzc;
    if (invzc < 0) continue;
    const float u = cam->fx * L.xc * invzc + cam->cx;
    const float v = cam->fy * L.yc * invzc + cam->cy;
    if (u < C->min_x || u > C->max_x) continue;
    if (v < C->min_y || v > C->max_y) continue;
    const int nLastOctave = L.last_octave;
    const float radius = th * C->scale_factors[nLastOctave];
    if (bForward) features_in_area(g, C->keys, u, v, radius, nLastOctave, -1, idxs);
    else if (bBackward) features_in_area(g, C->keys, u, v, radius, 0, nLastOctave, idxs);
    else features_in_area(g, C->keys, u, v, radius, nLastOctave - 1, nLastOctave + 1, idxs);
    if (idxs.empty()) continue;
    const uint8_t* d = last_desc + (size_t)i * 32;
    int bestDist = 256, bestIdx2 = -1;
    for (size_t i2 : idxs) {
      if (locked[i2]) continue;
      if (C->u_right && C->u_right[i2] > 0) {
        const float ur = u - cam->bf * invzc;
        const float er = fabsf(ur - C->u_right[i2]);
        if (er > radius) continue;
      }
      const int dist = descriptor_distance(d, C->descriptors + i2 * 32);
      if (dist < bestDist) { bestDist = dist; bestIdx2 = (int)i2; }
    }
    if (bestDist <= 100) {
      slot[bestIdx2] = L.mp_id;
      state[bestIdx2] = 1;
      locked[bestIdx2] = L.has_obs;
      ++nmatches;
      if (checkOri) rotHist[rot_bin(L.last_angle - C->keys[bestIdx2].angle)].push_back(bestIdx2);
    }
  }
  if (checkOri) {
    int ind1 = -1, ind2 = -1, ind3 = -1;
    three_maxima(rotHist, 30, ind1, ind2, ind3);
    for (int b = 0; b < 30; ++b) {
      if (b == ind1 || b == ind2 || b == ind3) continue;
      for (int idx : rotHist[b]) { slot[idx] = -1; state[idx] = 2; locked[idx] = 0; --nmatches; }
    }
  }
  // kp_match: MapPoint id assigned by this call, -1 untouched, -2 set to NULL by this call
  for (int i = 0; i < C->n; ++i) kp_match[i] = state[i] == 1 ? slot[i] : (state[i] == 2 ? -2 : -1);
  return nmatches;
}

// a17: SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&), src/ORBmatcher.cc:164-306
static int search_by_bow(int n_kf, const uint8_t* kf_desc, const float* kf_angle,
                         const int32_t* kf_mp, const uint8_t* kf_mp_bad, int kf_nodes,
                         const uint32_t* kf_node_ids, const int32_t* kf_offs,
                         const uint32_t* kf_feats, int n_f, const uint8_t* f_desc,
                         const float* f_angle, int f_nodes, const uint32_t* f_node_ids,
                         const int32_t* f_offs, const uint32_t* f_feats, float nnratio,
                         int checkOri, int32_t* f_match) {
  (void)n_kf;
  for (int j = 0; j < n_f; ++j) f_match[j] = -1;
  std::vector<int> rotHist[30];
  int nmatches = 0;
  int a = 0, b = 0;
  while (a < kf_nodes && b < f_nodes) {
    if (kf_node_ids[a] == f_node_ids[b]) {
      for (int p = kf_offs[a]; p < kf_offs[a + 1]; ++p) {
        const int realIdxKF = (int)kf_feats[p];
        const int mp = kf_mp[realIdxKF];
        if (mp < 0) continue;
        if (kf_mp_bad && kf_mp_bad[realIdxKF]) continue;
        const uint8_t* dKF = kf_desc + (size_t)realIdxKF * 32;
        int best1 = 256, bestIdxF = -1, best2 = 256;
        for (int q = f_offs[b]; q < f_offs[b + 1]; ++q) {
          const int realIdxF = (int)f_feats[q];
          if (f_match[realIdxF] >= 0) continue;
          const int dist = descriptor_distance(dKF, f_desc + (size_t)realIdxF * 32);
          if (dist < best1) { best2 = best1; best1 = dist; bestIdxF = realIdxF; }
          else if (dist < best2) best2 = dist;
        }
        if (best1 <= 50 && (float)best1 < nnratio * (float)best2) {
          f_match[bestIdxF] = mp;
          if (checkOri) rotHist[rot_bin(kf_angle[realIdxKF] - f_angle[bestIdxF])].push_back(bestIdxF);
          ++nmatches;
        }
      }
      ++a;
      ++b;
    } else if (kf_node_ids[a] < f_node_ids[b]) {
      a = (int)(std::lower_bound(kf_node_ids + a, kf_node_ids + kf_nodes, f_node_ids[b]) - kf_node_ids);
    } else {
      b = (int)(std::lower_bound(f_node_ids + b, f_node_ids + f_nodes, kf_node_ids[a]) - f_node_ids);
    }
  }
  if (checkOri) {
    int ind1 = -1, ind2 = -1, ind3 = -1;
    three_maxima(rotHist, 30, ind1, ind2, ind3);
    for (int bb = 0; bb < 30; ++bb) {
      if (bb == ind1 || bb == ind2 || bb == ind3) continue;
      for (int idx : rotHist[bb]) { f_match[idx] = -1; --nmatches; }
    }
  }
  return nmatches;
}

// a11: ComputeStereoMatches, src/Frame.cc:516-704 (debug ofstream of :556,652 omitted)
static void stereo_matches(const orb_stereo_input_t* in, float* uRight, float* depth) {
  const orb_frame_t* F = in->left;
  const int N = F->n;
  for (int i = 0; i < N; ++i) { uRight[i] = -1.0f; depth[i] = -1.0f; }
  const int thOrbDist = (100 + 50) / 2;
  const int nRows = in->level_height[0];
  std::vector<std::vector<size_t>> rowIdx(nRows);
  for (int iR = 0; iR < in->n_right; ++iR) {
    const orb_keypoint_t& kp = in->right_keys[iR];
    const float r = 2.0f * F->scale_factors[kp.octave];
    const int maxr = (int)ceilf(kp.y + r), minr = (int)floorf(kp.y - r);
    for (int yi = minr; yi <= maxr; ++yi) rowIdx[yi].push_back((size_t)iR);
  }
  const float mb = in->bf / in->fx;
  const float minZ = mb, minD = 0, maxD = in->bf / minZ;
  std::vector<std::pair<int, int>> distIdx;
  for (int iL = 0; iL < N; ++iL) {
    const orb_keypoint_t& kpL = F->keys[iL];
    const int levelL = kpL.octave;
    const float vL = kpL.y, uL = kpL.x;
    const std::vector<size_t>& cand = rowIdx[(size_t)vL];
    if (cand.empty()) continue;
    const float minU = uL - maxD, maxU = uL - minD;
    if (maxU < 0) continue;
    int bestDist = 100;
    size_t bestIdxR = 0;
    const uint8_t* dL = F->descriptors + (size_t)iL * 32;
    for (size_t iR : cand) {
      const orb_keypoint_t& kpR = in->right_keys[iR];
      if (kpR.octave < levelL - 1 || kpR.octave > levelL + 1) continue;
      const float uR = kpR.x;
      if (uR >= minU && uR <= maxU) {
        const int dist = descriptor_distance(dL, in->right_desc + iR * 32);
        if (dist < bestDist) { bestDist = dist; bestIdxR = iR; }
      }
    }
    if (bestDist < thOrbDist) {
      const float uR0 = in->right_keys[bestIdxR].x;
      const float scaleFactor = in->inv_scale_factors[kpL.octave];
      const float scaleduL = roundf(kpL.x * scaleFactor);
      const float scaledvL = roundf(kpL.y * scaleFactor);
      const float scaleduR0 = roundf(uR0 * scaleFactor);
      const int w = 5, L = 5;
      const int lw = in->level_width[levelL];
      const int64_t lsL = in->level_stride[levelL];
      const uint8_t* IL = in->left_levels[levelL];
      const uint8_t* IR = in->right_levels[levelL];
      const int ry0 = (int)scaledvL - w, lx0 = (int)scaleduL - w;
      const float iniu = scaleduR0 + L - w;
      const float endu = scaleduR0 + L + w + 1;
      if (iniu < 0 || endu >= lw) continue;
      const float cL = (float)IL[(int64_t)(ry0 + w) * lsL + lx0 + w];
      int bestSad = 2147483647;
      int bestincR = 0;
      float vDists[11];
      for (int incR = -L; incR <= L; ++incR) {
        const int rx0 = (int)scaleduR0 + incR - w;
        const float cR = (float)IR[(int64_t)(ry0 + w) * lsL + rx0 + w];
        float dist = 0.f;
        double acc = 0.0;
        for (int yy = 0; yy < 2 * w + 1; ++yy)
          for (int xx = 0; xx < 2 * w + 1; ++xx) {
            const float a = (float)IL[(int64_t)(ry0 + yy) * lsL + lx0 + xx] - cL;
            const float b = (float)IR[(int64_t)(ry0 + yy) * lsL + rx0 + xx] - cR;
            acc += fabs((double)a - (double)b);
          }
        dist = (float)acc;
        if (dist < bestSad) { bestSad = (int)dist; bestincR = incR; }
        vDists[L + incR] = dist;
      }
      if (bestincR == -L || bestincR == L) continue;
      const float dist1 = vDists[L + bestincR - 1], dist2 = vDists[L + bestincR],
                  dist3 = vDists[L + bestincR + 1];
      const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
      if (deltaR < -1 || deltaR > 1) continue;
      float bestuR = F->scale_factors[kpL.octave] * ((float)scaleduR0 + (float)bestincR + deltaR);
      float disparity = uL - bestuR;
      if (disparity >= minD && disparity < maxD) {
        if (disparity <= 0) { disparity = 0.01f; bestuR = (float)((double)uL - 0.01); }
        depth[iL] = in->bf / disparity;
        uRight[iL] = bestuR;
        distIdx.push_back(std::make_pair(bestSad, iL));
      }
    }
  }
  if (distIdx.empty()) return;  // reference indexes an empty vector here (UB)
  std::sort(distIdx.begin(), distIdx.end());
  const float median = (float)distIdx[distIdx.size() / 2].first;
  const float thDist = 1.5f * 1.4f * median;
  for (int i = (int)distIdx.size() - 1; i >= 0; --i) {
    if ((float)distIdx[i].first < thDist) break;
    uRight[distIdx[i].second] = -1;
    depth[distIdx[i].second] = -1;
  }
}

// f1: ORBmatcher::SearchForInitialization, src/ORBmatcher.cc:429-577.
// prev is vbPrevMatched as (x, y) pairs, updated in place; m12 = vnMatches12.
static int search_for_initialization(const orb_frame_t* F1, const orb_frame_t* F2, float* prev,
                                     int windowSize, float nnratio, int checkOri, int32_t* m12) {
  thread_local Grid g;  // per thread: the oracle runs on many host threads (bench.py cpu_all_cores)
  assign_grid(g, F2->keys, F2->n, F2->min_x, F2->max_x, F2->min_y, F2->max_y);
  const int N1 = F1->n, N2 = F2->n;
  int nmatches = 0;
  for (int i = 0; i < N1; ++i) m12[i] = -1;
  std::vector<int> rotHist[30];
  std::vector<int> matchedDist(N2, INT_MAX), m21(N2, -1);
  std::vector<size_t> cand;
  for (int i1 = 0; i1 < N1; ++i1) {
    const int level1 = F1->keys[i1].octave;
    if (level1 > 0) continue;                                            // :449-451
    features_in_area(g, F2->keys, prev[2 * i1], prev[2 * i1 + 1], (float)windowSize, level1,
                     level1, cand);                                       // :453
    if (cand.empty()) continue;
    const uint8_t* d1 = F1->descriptors + (size_t)i1 * 32;
    int bestDist = INT_MAX, bestDist2 = INT_MAX, bestIdx2 = -1;
    for (size_t i2 : cand) {                                              // :463-486
      const int dist = descriptor_distance(d1, F2->descriptors + i2 * 32);
      if (matchedDist[i2] <= dist) continue;
      if (dist < bestDist) {
        bestDist2 = bestDist;
        bestDist = dist;
        bestIdx2 = (int)i2;
      } else if (dist < bestDist2) {
        bestDist2 = dist;
      }
    }
    if (bestDist <= 50 && (float)bestDist < (float)bestDist2 * nnratio) {  // TH_LOW, :488-492
      if (m21[bestIdx2] >= 0) {  // steal: the earlier frame-1 point loses its match
        m12[m21[bestIdx2]] = -1;
        --nmatches;
      }
      m12[i1] = bestIdx2;
      m21[bestIdx2] = i1;
      matchedDist[bestIdx2] = bestDist;
      ++nmatches;
      if (checkOri) rotHist[rot_bin(F1->keys[i1].angle - F2->keys[bestIdx2].angle)].push_back(i1);
    }
  }
  if (checkOri) {                                                         // :540-568
    int ind1 = -1, ind2 = -1, ind3 = -1;
    three_maxima(rotHist, 30, ind1, ind2, ind3);
    for (int i = 0; i < 30; ++i) {
      if (i == ind1 || i == ind2 || i == ind3) continue;
      for (int idx1 : rotHist[i])
        if (m12[idx1] >= 0) {
          m12[idx1] = -1;
          --nmatches;
        }
    }
  }
  for (int i1 = 0; i1 < N1; ++i1)                                         // :571-574
    if (m12[i1] >= 0) {
      prev[2 * i1] = F2->keys[m12[i1]].x;
      prev[2 * i1 + 1] = F2->keys[m12[i1]].y;
    }
  return nmatches;
}

// f2: MapPoint::ComputeDistinctiveDescriptors, src/MapPoint.cc:250-326, for one
// point whose usable observation descriptors (observations in map order, bad
// KeyFrames dropped) are desc[0..n).  Returns BestIdx, or -1 when n == 0 (the
// reference returns without touching mDescriptor).
static int distinctive_descriptor(const uint8_t* desc, int n) {
  if (n <= 0) return -1;
  std::vector<int> D((size_t)n * n, 0);
  for (int i = 0; i < n; ++i)
    for (int j = i + 1; j < n; ++j)
      D[(size_t)i * n + j] = D[(size_t)j * n + i] =
          descriptor_distance(desc + (size_t)i * 32, desc + (size_t)j * 32);
  int bestMedian = INT_MAX, bestIdx = 0;
  std::vector<int> row(n);
  for (int i = 0; i < n; ++i) {
    row.assign(D.begin() + (size_t)i * n, D.begin() + (size_t)(i + 1) * n);
    std::sort(row.begin(), row.end());
    const int median = row[(size_t)(0.5 * (n - 1))];
    if (median < bestMedian) {
      bestMedian = median;
      bestIdx = i;
    }
  }
  return bestIdx;
}

// ------------------------------------------------------------------------
// §8(f) ORBmatcher variants.  Shared pinned arithmetic (parity unpinned: no
// reference fixture covers these; same cv::Mat pinning as frustum_one):
//   Mat*Mat (3x3 * 3x1) + Mat: float dot products left to right, then + t
//   scalar * Mat, Mat / scalar: (float)((double)x * alpha) with alpha double
//   Mat::dot, cv::norm: double accumulation; norm -> sqrt(double) -> float
//   -R^T t: float dot left to right, negated
struct Rt {
  float R[9], t[3], Ow[3];
};

static inline void xform(const float* R, const float* t, const float* P, float* out) {
  for (int r = 0; r < 3; ++r)
    out[r] = ((R[3 * r] * P[0] + R[3 * r + 1] * P[1]) + R[3 * r + 2] * P[2]) + t[r];
}

static inline void neg_rt_t(const float* R, const float* t, float* Ow) {
  for (int i = 0; i < 3; ++i) Ow[i] = -((R[i] * t[0] + R[3 + i] * t[1]) + R[6 + i] * t[2]);
}

// Scw (3x4, row-major [sR | st]) -> Rcw = sRcw/scw, tcw = st/scw, Ow = -Rcw^T tcw
// (src/ORBmatcher.cc:320-327, 1086-1092)
static Rt sim3_pose(const float* S) {
  Rt p;
  double ss = 0.0;
  for (int k = 0; k < 3; ++k) ss += (double)S[k] * S[k];
  const float scw = (float)sqrt(ss);
  const double inv = 1.0 / (double)scw;
  for (int r = 0; r < 3; ++r) {
    for (int c = 0; c < 3; ++c) p.R[3 * r + c] = (float)((double)S[4 * r + c] * inv);
    p.t[r] = (float)((double)S[4 * r + 3] * inv);
  }
  neg_rt_t(p.R, p.t, p.Ow);
  return p;
}

static inline float norm3(const float* a) {
  double ss = 0.0;
  for (int k = 0; k < 3; ++k) ss += (double)a[k] * a[k];
  return (float)sqrt(ss);
}

static inline double dot3(const float* a, const float* b) {
  double d = 0.0;
  for (int k = 0; k < 3; ++k) d += (double)a[k] * b[k];
  return d;
}

// MapPoint::PredictScale (src/MapPoint.cc:417-450), logf pinned
static inline int predict_scale(float maxDistance, float dist, float logScale, int nLevels) {
  const float ratio = maxDistance / dist;
  const float q = ceilf(scale_log(ratio) / logScale);
  if (q < 0.f) return 0;
  if (q >= (float)nLevels) return nLevels - 1;
  return (int)q;
}

static inline bool kf_in_image(const orb_frame_t* K, float x, float y) {  // KeyFrame::IsInImage
  return x >= K->min_x && x < K->max_x && y >= K->min_y && y < K->max_y;
}

// f4: SearchByProjection(Frame&, KeyFrame*, const set<MapPoint*>&, th, ORBdist),
// src/ORBmatcher.cc:1622-1759 (relocalisation).  Point i = the KeyFrame's map
// point of keypoint i (seen = in sAlreadyFound); kp_match[j] = point index
// assigned to frame keypoint j by this call, -2 reset by the rotation filter.
static int search_by_projection_reloc(const orb_frame_t* F, const uint8_t* kp_locked,
                                      const orb_pose_t* T, const orb_camera_t* cam,
                                      float logScale, int n, const orb_map_point_t* mps,
                                      const uint8_t* mpDesc, const float* kfAngle, float th,
                                      int orbDist, int checkOri, int32_t* kp_match) {
  thread_local Grid g;  // per thread: the oracle runs on many host threads (bench.py cpu_all_cores)
  assign_grid(g, F->keys, F->n, F->min_x, F->max_x, F->min_y, F->max_y);
  std::vector<uint8_t> locked(F->n, 0);
  for (int j = 0; j < F->n; ++j) {
    locked[j] = kp_locked ? kp_locked[j] : 0;
    kp_match[j] = -1;
  }
  std::vector<int> rotHist[30];
  std::vector<size_t> idxs;
  int nmatches = 0;
  for (int i = 0; i < n; ++i) {
    const orb_map_point_t& mp = mps[i];
    if (mp.bad || mp.seen) continue;
    float Pc[3];
    xform(T->rcw, T->tcw, mp.pos, Pc);
    const float invzc = (float)(1.0 / (double)Pc[2]);            // no z test here (:1660)
    const float u = cam->fx * Pc[0] * invzc + cam->cx;
    const float v = cam->fy * Pc[1] * invzc + cam->cy;
    if (u < F->min_x || u > F->max_x) continue;
    if (v < F->min_y || v > F->max_y) continue;
    const float PO[3] = {mp.pos[0] - T->ow[0], mp.pos[1] - T->ow[1], mp.pos[2] - T->ow[2]};
    const float dist3D = norm3(PO);
    if (dist3D < 0.8f * mp.min_distance || dist3D > 1.2f * mp.max_distance) continue;
    const int lvl = predict_scale(mp.max_distance, dist3D, logScale, F->n_levels);
    const float radius = th * F->scale_factors[lvl];
    features_in_area(g, F->keys, u, v, radius, lvl - 1, lvl + 1, idxs);
    if (idxs.empty()) continue;
    const uint8_t* dMP = mpDesc + (size_t)i * 32;
    int bestDist = 256, bestIdx = -1;
    for (size_t j : idxs) {
      if (locked[j]) continue;
      const int d = descriptor_distance(dMP, F->descriptors + j * 32);
      if (d < bestDist) { bestDist = d; bestIdx = (int)j; }
    }
    if (bestDist <= orbDist) {
      locked[bestIdx] = 1;
      kp_match[bestIdx] = i;
      ++nmatches;
      if (checkOri) rotHist[rot_bin(kfAngle[i] - F->keys[bestIdx].angle)].push_back(bestIdx);
    }
  }
  if (checkOri) {
    int ind1 = -1, ind2 = -1, ind3 = -1;
    three_maxima(rotHist, 30, ind1, ind2, ind3);
    for (int b = 0; b < 30; ++b) {
      if (b == ind1 || b == ind2 || b == ind3) continue;
      for (int j : rotHist[b]) { kp_match[j] = -2; --nmatches; }
    }
  }
  return nmatches;
}

// f5: SearchByProjection(KeyFrame*, Scw, vpPoints, vpMatched, th),
// src/ORBmatcher.cc:311-425 (loop closing).  kp_matched[j] = index of the
// point in vpMatched[j] or -1 (in/out); seen = in spAlreadyFound.
static int search_by_projection_sim3(const orb_frame_t* K, const float* Scw,
                                     const orb_camera_t* cam, float logScale, int n,
                                     const orb_map_point_t* mps, const uint8_t* mpDesc, float th,
                                     int32_t* kp_matched) {
  thread_local Grid g;  // per thread: the oracle runs on many host threads (bench.py cpu_all_cores)
  assign_grid(g, K->keys, K->n, K->min_x, K->max_x, K->min_y, K->max_y);
  const Rt T = sim3_pose(Scw);
  std::vector<size_t> idxs;
  int nmatches = 0;
  for (int i = 0; i < n; ++i) {
    const orb_map_point_t& mp = mps[i];
    if (mp.bad || mp.seen) continue;
    float Pc[3];
    xform(T.R, T.t, mp.pos, Pc);
    if (Pc[2] < 0.0) continue;
    const float invz = 1 / Pc[2];
    const float x = Pc[0] * invz, y = Pc[1] * invz;
    const float u = cam->fx * x + cam->cx, v = cam->fy * y + cam->cy;
    if (!kf_in_image(K, u, v)) continue;
    const float maxD = 1.2f * mp.max_distance, minD = 0.8f * mp.min_distance;
    const float PO[3] = {mp.pos[0] - T.Ow[0], mp.pos[1] - T.Ow[1], mp.pos[2] - T.Ow[2]};
    const float dist = norm3(PO);
    if (dist < minD || dist > maxD) continue;
    if (dot3(PO, mp.normal) < 0.5 * dist) continue;
    const int lvl = predict_scale(mp.max_distance, dist, logScale, K->n_levels);
    const float radius = th * K->scale_factors[lvl];
    features_in_area(g, K->keys, u, v, radius, -1, -1, idxs);
    if (idxs.empty()) continue;
    const uint8_t* dMP = mpDesc + (size_t)i * 32;
    int bestDist = 256, bestIdx = -1;
    for (size_t j : idxs) {
      if (kp_matched[j] >= 0) continue;
      const int kl = K->keys[j].octave;
      if (kl < lvl - 1 || kl > lvl) continue;
      const int d = descriptor_distance(dMP, K->descriptors + j * 32);
      if (d < bestDist) { bestDist = d; bestIdx = (int)j; }
    }
    if (bestDist <= 50) {
      kp_matched[bestIdx] = i;
      ++nmatches;
    }
  }
  return nmatches;
}

// f6: Fuse(KeyFrame*, vpMapPoints, th), src/ORBmatcher.cc:903-1077: the keypoint
// each point fuses into (best[i], -1 = none), from the state at entry; the
// Replace / AddObservation side effects stay with the caller (seen =
// IsInKeyFrame(pKF)).  Returns the number of points with a fuse target.
static int fuse_candidates(const orb_frame_t* K, const float* invSigma2, const orb_pose_t* T,
                           const orb_camera_t* cam, float logScale, int n,
                           const orb_map_point_t* mps, const uint8_t* mpDesc, float th,
                           int32_t* best) {
  thread_local Grid g;  // per thread: the oracle runs on many host threads (bench.py cpu_all_cores)
  assign_grid(g, K->keys, K->n, K->min_x, K->max_x, K->min_y, K->max_y);
  std::vector<size_t> idxs;
  int nf = 0;
  for (int i = 0; i < n; ++i) {
    best[i] = -1;
    const orb_map_point_t& mp = mps[i];
    if (mp.bad || mp.seen) continue;
    float Pc[3];
    xform(T->rcw, T->tcw, mp.pos, Pc);
    if (Pc[2] < 0.0f) continue;
    const float invz = 1 / Pc[2];
    const float x = Pc[0] * invz, y = Pc[1] * invz;
    const float u = cam->fx * x + cam->cx, v = cam->fy * y + cam->cy;
    if (!kf_in_image(K, u, v)) continue;
    const float ur = u - cam->bf * invz;
    const float maxD = 1.2f * mp.max_distance, minD = 0.8f * mp.min_distance;
    const float PO[3] = {mp.pos[0] - T->ow[0], mp.pos[1] - T->ow[1], mp.pos[2] - T->ow[2]};
    const float dist3D = norm3(PO);
    if (dist3D < minD || dist3D > maxD) continue;
    if (dot3(PO, mp.normal) < 0.5 * dist3D) continue;
    const int lvl = predict_scale(mp.max_distance, dist3D, logScale, K->n_levels);
    const float radius = th * K->scale_factors[lvl];
    features_in_area(g, K->keys, u, v, radius, -1, -1, idxs);
    if (idxs.empty()) continue;
    const uint8_t* dMP = mpDesc + (size_t)i * 32;
    int bestDist = 256, bestIdx = -1;
    for (size_t j : idxs) {
      const KP& kp = K->keys[j];
      const int kl = kp.octave;
      if (kl < lvl - 1 || kl > lvl) continue;
      if (K->u_right && K->u_right[j] >= 0) {
        const float ex = u - kp.x, ey = v - kp.y, er = ur - K->u_right[j];
        const float e2 = ex * ex + ey * ey + er * er;
        if (e2 * invSigma2[kl] > 7.8) continue;
      } else {
        const float ex = u - kp.x, ey = v - kp.y;
        const float e2 = ex * ex + ey * ey;
        if (e2 * invSigma2[kl] > 5.99) continue;
      }
      const int d = descriptor_distance(dMP, K->descriptors + j * 32);
      if (d < bestDist) { bestDist = d; bestIdx = (int)j; }
    }
    if (bestDist <= 50) {
      best[i] = bestIdx;
      ++nf;
    }
  }
  return nf;
}

// f7: Fuse(KeyFrame*, Scw, vpPoints, th, vpReplacePoint), src/ORBmatcher.cc:1079-1210:
// fuse target per point from the state at entry (seen = in spAlreadyFound).
static int fuse_sim3_candidates(const orb_frame_t* K, const float* Scw, const orb_camera_t* cam,
                                float logScale, int n, const orb_map_point_t* mps,
                                const uint8_t* mpDesc, float th, int32_t* best) {
  thread_local Grid g;  // per thread: the oracle runs on many host threads (bench.py cpu_all_cores)
  assign_grid(g, K->keys, K->n, K->min_x, K->max_x, K->min_y, K->max_y);
  const Rt T = sim3_pose(Scw);
  std::vector<size_t> idxs;
  int nf = 0;
  for (int i = 0; i < n; ++i) {
    best[i] = -1;
    const orb_map_point_t& mp = mps[i];
    if (mp.bad || mp.seen) continue;
    float Pc[3];
    xform(T.R, T.t, mp.pos, Pc);
    if (Pc[2] < 0.0f) continue;
    const float invz = (float)(1.0 / (double)Pc[2]);
    const float x = Pc[0] * invz, y = Pc[1] * invz;
    const float u = cam->fx * x + cam->cx, v = cam->fy * y + cam->cy;
    if (!kf_in_image(K, u, v)) continue;
    const float maxD = 1.2f * mp.max_distance, minD = 0.8f * mp.min_distance;
    const float PO[3] = {mp.pos[0] - T.Ow[0], mp.pos[1] - T.Ow[1], mp.pos[2] - T.Ow[2]};
    const float dist3D = norm3(PO);
    if (dist3D < minD || dist3D > maxD) continue;
    if (dot3(PO, mp.normal) < 0.5 * dist3D) continue;
    const int lvl = predict_scale(mp.max_distance, dist3D, logScale, K->n_levels);
    const float radius = th * K->scale_factors[lvl];
    features_in_area(g, K->keys, u, v, radius, -1, -1, idxs);
    if (idxs.empty()) continue;
    const uint8_t* dMP = mpDesc + (size_t)i * 32;
    int bestDist = INT_MAX, bestIdx = -1;
    for (size_t j : idxs) {
      const int kl = K->keys[j].octave;
      if (kl < lvl - 1 || kl > lvl) continue;
      const int d = descriptor_distance(dMP, K->descriptors + j * 32);
      if (d < bestDist) { bestDist = d; bestIdx = (int)j; }
    }
    if (bestDist <= 50) {
      best[i] = bestIdx;
      ++nf;
    }
  }
  return nf;
}

// One direction of SearchBySim3 (src/ORBmatcher.cc:1256-1330 / 1332-1404):
// points of keyframe A (pose RAw, tAw) through the similarity (sR, t) into
// keyframe B; out[i] = best B keypoint (<= TH_HIGH) or -1.
static void sim3_direction(const orb_frame_t* B, float logScaleB, const orb_camera_t* cam,
                           const float* RAw, const float* tAw, const float* sR, const float* t,
                           int nA, const orb_map_point_t* mpsA, const uint8_t* validA,
                           const uint8_t* alreadyA, const uint8_t* descA, float th,
                           int32_t* out) {
  thread_local Grid g;  // per thread: the oracle runs on many host threads (bench.py cpu_all_cores)
  assign_grid(g, B->keys, B->n, B->min_x, B->max_x, B->min_y, B->max_y);
  std::vector<size_t> idxs;
  for (int i = 0; i < nA; ++i) {
    out[i] = -1;
    if (!validA[i] || alreadyA[i]) continue;
    const orb_map_point_t& mp = mpsA[i];
    if (mp.bad) continue;
    float Pa[3], Pb[3];
    xform(RAw, tAw, mp.pos, Pa);
    xform(sR, t, Pa, Pb);
    if (Pb[2] < 0.0) continue;
    const float invz = (float)(1.0 / (double)Pb[2]);
    const float x = Pb[0] * invz, y = Pb[1] * invz;
    const float u = cam->fx * x + cam->cx, v = cam->fy * y + cam->cy;
    if (!kf_in_image(B, u, v)) continue;
    const float maxD = 1.2f * mp.max_distance, minD = 0.8f * mp.min_distance;
    const float dist3D = norm3(Pb);
    if (dist3D < minD || dist3D > maxD) continue;
    const int lvl = predict_scale(mp.max_distance, dist3D, logScaleB, B->n_levels);
    const float radius = th * B->scale_factors[lvl];
    features_in_area(g, B->keys, u, v, radius, -1, -1, idxs);
    if (idxs.empty()) continue;
    const uint8_t* dMP = descA + (size_t)i * 32;
    int bestDist = INT_MAX, bestIdx = -1;
    for (size_t j : idxs) {
      const int kl = B->keys[j].octave;
      if (kl < lvl - 1 || kl > lvl) continue;
      const int d = descriptor_distance(dMP, B->descriptors + j * 32);
      if (d < bestDist) { bestDist = d; bestIdx = (int)j; }
    }
    if (bestDist <= 100) out[i] = bestIdx;
  }
}

// f8: SearchBySim3, src/ORBmatcher.cc:1212-1458.  match12[i1] = idx2 of a
// mutual match (vpMatches12[i1] = vpMapPoints2[idx2]) or -1.
static int search_by_sim3(const orb_frame_t* K1, const orb_frame_t* K2, float logScale1,
                          float logScale2, const orb_camera_t* cam, const float* R1w,
                          const float* t1w, const float* R2w, const float* t2w,
                          const orb_map_point_t* mps1, const uint8_t* valid1,
                          const uint8_t* already1, const uint8_t* mpDesc1,
                          const orb_map_point_t* mps2, const uint8_t* valid2,
                          const uint8_t* already2, const uint8_t* mpDesc2, float s12,
                          const float* R12, const float* t12, float th, int32_t* match12) {
  float sR12[9], sR21[9], t21[3];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) {
      sR12[3 * r + c] = (float)((double)s12 * (double)R12[3 * r + c]);
      sR21[3 * r + c] = (float)((1.0 / (double)s12) * (double)R12[3 * c + r]);
    }
  for (int r = 0; r < 3; ++r)
    t21[r] = -((sR21[3 * r] * t12[0] + sR21[3 * r + 1] * t12[1]) + sR21[3 * r + 2] * t12[2]);
  std::vector<int32_t> m1(K1->n), m2(K2->n);
  sim3_direction(K2, logScale2, cam, R1w, t1w, sR21, t21, K1->n, mps1, valid1, already1,
                 mpDesc1, th, m1.data());
  sim3_direction(K1, logScale1, cam, R2w, t2w, sR12, t12, K2->n, mps2, valid2, already2,
                 mpDesc2, th, m2.data());
  int nFound = 0;
  for (int i1 = 0; i1 < K1->n; ++i1) {
    match12[i1] = -1;
    const int idx2 = m1[i1];
    if (idx2 >= 0 && m2[idx2] == i1) {
      match12[i1] = idx2;
      ++nFound;
    }
  }
  return nFound;
}

// f9: SearchByBoW(KeyFrame*, KeyFrame*, vpMatches12), src/ORBmatcher.cc:581-716.
// match12[idx1] = MapPoint id of the matched KF2 keypoint or -1.
static int search_by_bow_kf(const uint8_t* d1, const float* a1, const int32_t* mp1,
                            const uint8_t* bad1, int n1, int nodes1, const uint32_t* ids1,
                            const int32_t* offs1, const uint32_t* feats1, const uint8_t* d2,
                            const float* a2, const int32_t* mp2, const uint8_t* bad2, int n2,
                            int nodes2, const uint32_t* ids2, const int32_t* offs2,
                            const uint32_t* feats2, float nnratio, int checkOri,
                            int32_t* match12) {
  for (int i = 0; i < n1; ++i) match12[i] = -1;
  std::vector<uint8_t> matched2(n2, 0);
  std::vector<int> rotHist[30];
  int nmatches = 0;
  int a = 0, b = 0;
  while (a < nodes1 && b < nodes2) {
    if (ids1[a] == ids2[b]) {
      for (int p = offs1[a]; p < offs1[a + 1]; ++p) {
        const int idx1 = (int)feats1[p];
        if (mp1[idx1] < 0 || (bad1 && bad1[idx1])) continue;
        int best1 = 256, bestIdx2 = -1, best2 = 256;
        for (int q = offs2[b]; q < offs2[b + 1]; ++q) {
          const int idx2 = (int)feats2[q];
          if (matched2[idx2] || mp2[idx2] < 0) continue;
          if (bad2 && bad2[idx2]) continue;
          const int dist = descriptor_distance(d1 + (size_t)idx1 * 32, d2 + (size_t)idx2 * 32);
          if (dist < best1) { best2 = best1; best1 = dist; bestIdx2 = idx2; }
          else if (dist < best2) best2 = dist;
        }
        if (best1 < 50 && (float)best1 < nnratio * (float)best2) {  // TH_LOW strict (:650)
          match12[idx1] = mp2[bestIdx2];
          matched2[bestIdx2] = 1;
          if (checkOri) rotHist[rot_bin(a1[idx1] - a2[bestIdx2])].push_back(idx1);
          ++nmatches;
        }
      }
      ++a;
      ++b;
    } else if (ids1[a] < ids2[b]) {
      a = (int)(std::lower_bound(ids1 + a, ids1 + nodes1, ids2[b]) - ids1);
    } else {
      b = (int)(std::lower_bound(ids2 + b, ids2 + nodes2, ids1[a]) - ids2);
    }
  }
  if (checkOri) {
    int ind1 = -1, ind2 = -1, ind3 = -1;
    three_maxima(rotHist, 30, ind1, ind2, ind3);
    for (int bb = 0; bb < 30; ++bb) {
      if (bb == ind1 || bb == ind2 || bb == ind3) continue;
      for (int idx : rotHist[bb]) { match12[idx] = -1; --nmatches; }
    }
  }
  return nmatches;
}

// CheckDistEpipolarLine, src/ORBmatcher.cc:144-161 (3.84 is a double literal)
static inline bool epipolar_ok(const KP& k1, const KP& k2, const float* F, float sigma2) {
  const float a = k1.x * F[0] + k1.y * F[3] + F[6];
  const float b = k1.x * F[1] + k1.y * F[4] + F[7];
  const float c = k1.x * F[2] + k1.y * F[5] + F[8];
  const float num = a * k2.x + b * k2.y + c;
  const float den = a * a + b * b;
  if (den == 0) return false;
  const float dsqr = num * num / den;
  return dsqr < 3.84 * sigma2;
}

// f10: SearchForTriangulation, src/ORBmatcher.cc:718-901.  Note the fork (as
// upstream) never sets vbMatched2, so idx1 queries are independent; among the
// passing candidates the LAST one with the smallest distance wins (<=).
// Epipole (ex, ey) from C2 = R2w*Cw + t2w (:728-733).
static int search_for_triangulation(const orb_frame_t* K1, const uint8_t* has_mp1,
                                    const orb_frame_t* K2, const uint8_t* has_mp2,
                                    const float* levelSigma2, const float* F12,
                                    const orb_camera_t* cam, const float* Cw, const float* R2w,
                                    const float* t2w, int nodes1, const uint32_t* ids1,
                                    const int32_t* offs1, const uint32_t* feats1, int nodes2,
                                    const uint32_t* ids2, const int32_t* offs2,
                                    const uint32_t* feats2, int onlyStereo, int checkOri,
                                    int32_t* match12) {
  float C2[3];
  xform(R2w, t2w, Cw, C2);
  const float invz = 1.0f / C2[2];
  const float ex = cam->fx * C2[0] * invz + cam->cx;
  const float ey = cam->fy * C2[1] * invz + cam->cy;
  for (int i = 0; i < K1->n; ++i) match12[i] = -1;
  std::vector<int> rotHist[30];
  int nmatches = 0;
  int a = 0, b = 0;
  while (a < nodes1 && b < nodes2) {
    if (ids1[a] == ids2[b]) {
      for (int p = offs1[a]; p < offs1[a + 1]; ++p) {
        const int idx1 = (int)feats1[p];
        if (has_mp1[idx1]) continue;
        const bool st1 = K1->u_right && K1->u_right[idx1] >= 0;
        if (onlyStereo && !st1) continue;
        const KP& kp1 = K1->keys[idx1];
        const uint8_t* d1 = K1->descriptors + (size_t)idx1 * 32;
        int bestDist = 50, bestIdx2 = -1;
        for (int q = offs2[b]; q < offs2[b + 1]; ++q) {
          const int idx2 = (int)feats2[q];
          if (has_mp2[idx2]) continue;  // vbMatched2 is never set (:785)
          const bool st2 = K2->u_right && K2->u_right[idx2] >= 0;
          if (onlyStereo && !st2) continue;
          const int dist = descriptor_distance(d1, K2->descriptors + (size_t)idx2 * 32);
          if (dist > 50 || dist > bestDist) continue;
          const KP& kp2 = K2->keys[idx2];
          if (!st1 && !st2) {
            const float dx = ex - kp2.x, dy = ey - kp2.y;
            if (dx * dx + dy * dy < 100 * K2->scale_factors[kp2.octave]) continue;
          }
          if (epipolar_ok(kp1, kp2, F12, levelSigma2[kp2.octave])) {
            bestIdx2 = idx2;
            bestDist = dist;
          }
        }
        if (bestIdx2 >= 0) {
          match12[idx1] = bestIdx2;
          ++nmatches;
          if (checkOri) rotHist[rot_bin(kp1.angle - K2->keys[bestIdx2].angle)].push_back(idx1);
        }
      }
      ++a;
      ++b;
    } else if (ids1[a] < ids2[b]) {
      a = (int)(std::lower_bound(ids1 + a, ids1 + nodes1, ids2[b]) - ids1);
    } else {
      b = (int)(std::lower_bound(ids2 + b, ids2 + nodes2, ids1[a]) - ids2);
    }
  }
  if (checkOri) {
    int ind1 = -1, ind2 = -1, ind3 = -1;
    three_maxima(rotHist, 30, ind1, ind2, ind3);
    for (int bb = 0; bb < 30; ++bb) {
      if (bb == ind1 || bb == ind2 || bb == ind3) continue;
      for (int idx : rotHist[bb]) { match12[idx] = -1; --nmatches; }
    }
  }
  return nmatches;
}

}  // namespace oracle

// ===================================================================== C API
using namespace oracle;

extern "C" {

int oracle_params(int nfeatures, float scaleFactor, int nlevels, float* scale, float* inv_scale,
                  float* sigma2, float* inv_sigma2, int32_t* quota, int32_t* umax16) {
  const Params p = make_params(nfeatures, scaleFactor, nlevels, 20, 7);
  for (int l = 0; l < nlevels; ++l) {
    if (scale) scale[l] = p.scale[l];
    if (inv_scale) inv_scale[l] = p.invScale[l];
    if (sigma2) sigma2[l] = p.sigma2[l];
    if (inv_sigma2) inv_sigma2[l] = p.invSigma2[l];
    if (quota) quota[l] = p.quota[l];
  }
  if (umax16) for (int v = 0; v < 16; ++v) umax16[v] = p.umax[v];
  return 0;
}

static Img to_img(const uint8_t* img, int w, int h, size_t stride) {
  Img im(w, h);
  for (int y = 0; y < h; ++y) memcpy(im.row(y), img + (size_t)y * stride, (size_t)w);
  return im;
}

// Level sizes of the pyramid (2*nlevels ints: w0,h0,w1,h1,...).
int oracle_level_sizes(int w, int h, float scaleFactor, int nlevels, int32_t* wh) {
  const Params p = make_params(1000, scaleFactor, nlevels, 20, 7);
  for (int l = 0; l < nlevels; ++l) {
    wh[2 * l] = l ? cvRound((float)w * p.invScale[l]) : w;
    wh[2 * l + 1] = l ? cvRound((float)h * p.invScale[l]) : h;
  }
  return 0;
}

// Pyramid levels packed tightly level after level into `out`.
int oracle_pyramid(const uint8_t* img, int w, int h, size_t stride, float scaleFactor,
                   int nlevels, uint8_t* out) {
  const Params p = make_params(1000, scaleFactor, nlevels, 20, 7);
  const std::vector<Img> pyr = compute_pyramid(p, to_img(img, w, h, stride));
  size_t off = 0;
  for (const Img& l : pyr) {
    memcpy(out + off, l.px.data(), l.px.size());
    off += l.px.size();
  }
  return (int)off;
}

int oracle_resize(const uint8_t* src, int sw, int sh, uint8_t* dst, int dw, int dh) {
  const Img d = resize_linear(to_img(src, sw, sh, (size_t)sw), dw, dh);
  memcpy(dst, d.px.data(), d.px.size());
  return 0;
}

int oracle_blur7(const uint8_t* src, int w, int h, uint8_t* dst) {
  const Img d = gaussian_blur7(to_img(src, w, h, (size_t)w));
  memcpy(dst, d.px.data(), d.px.size());
  return 0;
}

// cv::FAST(img, kps, threshold, true) on a whole (small) image.
int oracle_fast(const uint8_t* img, int w, int h, int threshold, orb_keypoint_t* out, int cap) {
  std::vector<KP> kps;
  fast_roi(to_img(img, w, h, (size_t)w), 0, h, 0, w, threshold, kps);
  const int n = (int)kps.size();
  for (int i = 0; i < n && i < cap; ++i) out[i] = kps[i];
  return n;
}

float oracle_fast_atan2(float y, float x) { return fast_atan2(y, x); }

void oracle_sincos(float angle, float* s, float* c) { desc_sincos(angle, s, c); }

int oracle_descriptor_distance(const uint8_t* a, const uint8_t* b) { return descriptor_distance(a, b); }

// Per-level FAST candidates (vToDistributeKeys) of an image: writes up to cap
// keys (relative to the border origin, octave = level) and per-level counts.
int oracle_candidates(const uint8_t* img, int w, int h, size_t stride, int nfeatures,
                      float scaleFactor, int nlevels, int iniTh, int minTh, orb_keypoint_t* out,
                      int cap, int32_t* per_level) {
  const Params p = make_params(nfeatures, scaleFactor, nlevels, iniTh, minTh);
  const std::vector<Img> pyr = compute_pyramid(p, to_img(img, w, h, stride));
  int n = 0;
  std::vector<KP> cand;
  for (int l = 0; l < nlevels; ++l) {
    level_candidates(p, pyr[l], cand);
    per_level[l] = (int)cand.size();
    for (KP k : cand) {
      k.octave = l;
      if (n < cap) out[n] = k;
      ++n;
    }
  }
  return n;
}

// DistributeOctTree on an explicit key list (keys relative to the border origin).
int oracle_distribute(const orb_keypoint_t* keys, int n, int minX, int maxX, int minY, int maxY,
                      int N, orb_keypoint_t* out, int cap) {
  std::vector<KP> in(keys, keys + n);
  std::vector<KP> res = distribute_oct_tree(in, minX, maxX, minY, maxY, N);
  for (int i = 0; i < (int)res.size() && i < cap; ++i) out[i] = res[i];
  return (int)res.size();
}

// Full ORBextractor::operator(): returns N (or -N-1 if cap too small).
int oracle_extract(const uint8_t* img, int w, int h, size_t stride, int nfeatures,
                   float scaleFactor, int nlevels, int iniTh, int minTh, orb_keypoint_t* kps,
                   uint8_t* desc, int cap, int32_t* per_level) {
  const Params p = make_params(nfeatures, scaleFactor, nlevels, iniTh, minTh);
  ExtractResult r;
  extract(p, to_img(img, w, h, stride), r);
  const int n = (int)r.keys.size();
  if (per_level) for (int l = 0; l < nlevels; ++l) per_level[l] = r.perLevel[l];
  if (n > cap) return -n - 1;
  memcpy(kps, r.keys.data(), (size_t)n * sizeof(KP));
  memcpy(desc, r.desc.data(), (size_t)n * 32);
  return n;
}

int oracle_match_projection_local(const orb_frame_t* F, const uint8_t* kp_locked, int nmp,
                                  const orb_mp_track_t* mps, const uint8_t* mp_desc, float th,
                                  float nnratio, int32_t* kp_match) {
  return search_by_projection_local(F, kp_locked, nmp, mps, mp_desc, th, nnratio, kp_match);
}

double oracle_log(double x) { return pinned_log(x); }

int oracle_frustum(int n, const orb_map_point_t* mps, const orb_pose_t* pose,
                   const orb_camera_t* cam, float minX, float maxX, float minY, float maxY,
                   float cosLimit, float logScale, int nLevels, orb_mp_track_t* tracks) {
  FrustumCfg c;
  c.cam = *cam;
  c.minX = minX;
  c.maxX = maxX;
  c.minY = minY;
  c.maxY = maxY;
  c.cosLimit = cosLimit;
  c.logScale = logScale;
  c.nLevels = nLevels;
  return frustum_all(n, mps, *pose, c, tracks);
}

int oracle_match_projection_frame(const orb_frame_t* C, const uint8_t* kp_locked, int nlast,
                                  const orb_last_mp_t* last, const uint8_t* last_desc,
                                  const orb_camera_t* cam, float tlc_z, float th, int mono,
                                  int checkOri, int32_t* kp_match) {
  return search_by_projection_frame(C, kp_locked, nlast, last, last_desc, cam, tlc_z, th, mono,
                                    checkOri, kp_match);
}

int oracle_match_bow(int n_kf, const uint8_t* kf_desc, const float* kf_angle,
                     const int32_t* kf_mp, const uint8_t* kf_mp_bad, int kf_nodes,
                     const uint32_t* kf_node_ids, const int32_t* kf_offs,
                     const uint32_t* kf_feats, int n_f, const uint8_t* f_desc,
                     const float* f_angle, int f_nodes, const uint32_t* f_node_ids,
                     const int32_t* f_offs, const uint32_t* f_feats, float nnratio,
                     int check_orientation, int32_t* f_match) {
  return search_by_bow(n_kf, kf_desc, kf_angle, kf_mp, kf_mp_bad, kf_nodes, kf_node_ids,
                       kf_offs, kf_feats, n_f, f_desc, f_angle, f_nodes, f_node_ids, f_offs,
                       f_feats, nnratio, check_orientation, f_match);
}

int oracle_search_for_initialization(const orb_frame_t* F1, const orb_frame_t* F2, float* prev,
                                     int window_size, float nnratio, int check_orientation,
                                     int32_t* matches12) {
  return search_for_initialization(F1, F2, prev, window_size, nnratio, check_orientation,
                                   matches12);
}

// best[p] = BestIdx of point p over desc[offs[p]..offs[p+1]) (-1 when empty)
void oracle_distinctive_descriptors(int n_mp, const int32_t* offs, const uint8_t* desc,
                                    int32_t* best) {
  for (int p = 0; p < n_mp; ++p)
    best[p] = distinctive_descriptor(desc + (size_t)offs[p] * 32, offs[p + 1] - offs[p]);
}

int oracle_search_by_projection_reloc(const orb_frame_t* F, const uint8_t* kp_locked,
                                      const orb_pose_t* T, const orb_camera_t* cam,
                                      float log_scale, int n, const orb_map_point_t* mps,
                                      const uint8_t* mp_desc, const float* kf_angle, float th,
                                      int orb_dist, int check_ori, int32_t* kp_match) {
  return search_by_projection_reloc(F, kp_locked, T, cam, log_scale, n, mps, mp_desc, kf_angle,
                                    th, orb_dist, check_ori, kp_match);
}

int oracle_search_by_projection_sim3(const orb_frame_t* K, const float* scw,
                                     const orb_camera_t* cam, float log_scale, int n,
                                     const orb_map_point_t* mps, const uint8_t* mp_desc, float th,
                                     int32_t* kp_matched) {
  return search_by_projection_sim3(K, scw, cam, log_scale, n, mps, mp_desc, th, kp_matched);
}

int oracle_fuse(const orb_frame_t* K, const float* inv_sigma2, const orb_pose_t* T,
                const orb_camera_t* cam, float log_scale, int n, const orb_map_point_t* mps,
                const uint8_t* mp_desc, float th, int32_t* best) {
  return fuse_candidates(K, inv_sigma2, T, cam, log_scale, n, mps, mp_desc, th, best);
}

int oracle_fuse_sim3(const orb_frame_t* K, const float* scw, const orb_camera_t* cam,
                     float log_scale, int n, const orb_map_point_t* mps, const uint8_t* mp_desc,
                     float th, int32_t* best) {
  return fuse_sim3_candidates(K, scw, cam, log_scale, n, mps, mp_desc, th, best);
}

int oracle_search_by_sim3(const orb_frame_t* K1, const orb_frame_t* K2, float log_scale1,
                          float log_scale2, const orb_camera_t* cam, const float* R1w,
                          const float* t1w, const float* R2w, const float* t2w,
                          const orb_map_point_t* mps1, const uint8_t* valid1,
                          const uint8_t* already1, const uint8_t* mp_desc1,
                          const orb_map_point_t* mps2, const uint8_t* valid2,
                          const uint8_t* already2, const uint8_t* mp_desc2, float s12,
                          const float* R12, const float* t12, float th, int32_t* match12) {
  return search_by_sim3(K1, K2, log_scale1, log_scale2, cam, R1w, t1w, R2w, t2w, mps1, valid1,
                        already1, mp_desc1, mps2, valid2, already2, mp_desc2, s12, R12, t12, th,
                        match12);
}

int oracle_search_by_bow_kf(const uint8_t* d1, const float* a1, const int32_t* mp1,
                            const uint8_t* bad1, int n1, int nodes1, const uint32_t* ids1,
                            const int32_t* offs1, const uint32_t* feats1, const uint8_t* d2,
                            const float* a2, const int32_t* mp2, const uint8_t* bad2, int n2,
                            int nodes2, const uint32_t* ids2, const int32_t* offs2,
                            const uint32_t* feats2, float nnratio, int check_ori,
                            int32_t* match12) {
  return search_by_bow_kf(d1, a1, mp1, bad1, n1, nodes1, ids1, offs1, feats1, d2, a2, mp2, bad2,
                          n2, nodes2, ids2, offs2, feats2, nnratio, check_ori, match12);
}

int oracle_search_for_triangulation(const orb_frame_t* K1, const uint8_t* has_mp1,
                                    const orb_frame_t* K2, const uint8_t* has_mp2,
                                    const float* level_sigma2, const float* F12,
                                    const orb_camera_t* cam, const float* Cw, const float* R2w,
                                    const float* t2w, int nodes1, const uint32_t* ids1,
                                    const int32_t* offs1, const uint32_t* feats1, int nodes2,
                                    const uint32_t* ids2, const int32_t* offs2,
                                    const uint32_t* feats2, int only_stereo, int check_ori,
                                    int32_t* match12) {
  return search_for_triangulation(K1, has_mp1, K2, has_mp2, level_sigma2, F12, cam, Cw, R2w, t2w,
                                  nodes1, ids1, offs1, feats1, nodes2, ids2, offs2, feats2,
                                  only_stereo, check_ori, match12);
}

int oracle_stereo_match(const orb_stereo_input_t* in, float* u_right, float* depth) {
  stereo_matches(in, u_right, depth);
  return 0;
}

// Grid CSR of a frame: cell_start[64*48+1] (cell index = ix*48 + iy), idx[].
int oracle_grid(const orb_keypoint_t* keys, int n, float minX, float maxX, float minY,
                float maxY, int32_t* cell_start, int32_t* idx) {
  thread_local Grid g;  // per thread: the oracle runs on many host threads (bench.py cpu_all_cores)
  assign_grid(g, keys, n, minX, maxX, minY, maxY);
  int off = 0;
  for (int ix = 0; ix < ORB_GRID_COLS; ++ix)
    for (int iy = 0; iy < ORB_GRID_ROWS; ++iy) {
      cell_start[ix * ORB_GRID_ROWS + iy] = off;
      for (size_t k : g.cell[ix][iy]) idx[off++] = (int32_t)k;
    }
  cell_start[ORB_GRID_COLS * ORB_GRID_ROWS] = off;
  return off;
}

void oracle_synth_image(uint64_t seed, int frame, int view, int w, int h, uint8_t* out,
                        size_t stride) {
  orb_synth::render(seed, frame, view, w, h, out, stride);
}

void oracle_synth_local_map(uint64_t seed, const orb_keypoint_t* keys, const uint8_t* desc,
                            int n_kp, int n_mp, int w, int h, orb_mp_track_t* mps,
                            uint8_t* mp_desc, uint8_t* kp_locked) {
  orb_synth::local_map(seed, keys, desc, n_kp, n_mp, w, h, mps, mp_desc, kp_locked);
}

}  // extern "C"
