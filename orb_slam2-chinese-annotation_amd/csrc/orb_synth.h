// orb_synth.h -- deterministic synthetic inputs (header-only, integer arithmetic only).
//
// Inputs, not algorithm: KITTI/TUM sequences are not available offline
// (SURVEY.md §7 H8), so every benchmark config and parity test draws images
// and local maps from this generator (recipe: SURVEY.md §8(d)).  Integer-only
// so that the g++-built oracle and the hipcc-built library produce identical
// bytes for the same seed.
#pragma once
#include <stdint.h>
#include <stddef.h>
#include <string.h>

#include "../../include/orb_abi.h"

namespace orb_synth {

static inline uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct Rng {  // splitmix64 stream
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed) {}
  uint64_t next() { s += 0x9E3779B97F4A7C15ull; return mix64(s); }
  uint32_t below(uint32_t n) { return (uint32_t)(next() % n); }
};

struct Shape {
  int kind, cx, cy, hw, hh, val, disp;
};

// Cumulative horizontal ego-motion in pixels before frame `frame` (dx in U{-3..3}).
static inline int ego_offset(uint64_t seed, int frame) {
  int off = 0;
  for (int k = 0; k < frame; ++k) off += (int)(mix64(seed ^ (0xE6000000ull + (uint64_t)k)) % 7) - 3;
  return off;
}

static inline void render(uint64_t seed, int frame, int view, int W, int H, uint8_t* out,
                          size_t stride) {
  Rng r(seed * 0x2545F4914F6CDD1Dull + 0x5EEDull);
  const int c0 = 60 + (int)r.below(136);
  const int gx = (int)r.below(241) - 120;  // intensity change per 1024 px
  const int gy = (int)r.below(241) - 120;
  const long area = (long)W * H;
  int n = 300 + (int)r.below(501);
  if (area > 640L * 480L) n = (int)((long)n * area / (640L * 480L));
  const int margin = 40;
  const int maxHalf = 3 + (W < H ? W : H) / 10;

  // shapes, painted far (small disparity) to near; stable on index
  Shape* sh = new Shape[n];
  for (int i = 0; i < n; ++i) {
    Shape& s = sh[i];
    s.kind = (int)(r.next() & 1);
    s.cx = (int)r.below((uint32_t)(W + 2 * margin)) - margin;
    s.cy = (int)r.below((uint32_t)(H + 2 * margin)) - margin;
    s.hw = 2 + (int)r.below((uint32_t)maxHalf);
    s.hh = 2 + (int)r.below((uint32_t)maxHalf);
    s.val = (int)r.below(256);
    s.disp = 5 + (int)r.below(56);
  }
  for (int i = 1; i < n; ++i) {  // insertion sort by disparity (stable)
    Shape t = sh[i];
    int j = i - 1;
    while (j >= 0 && sh[j].disp > t.disp) { sh[j + 1] = sh[j]; --j; }
    sh[j + 1] = t;
  }

  // background gradient
  int* buf = new int[(size_t)W * H];
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) buf[(size_t)y * W + x] = c0 + (gx * x + gy * y) / 1024;

  const int ox = ego_offset(seed, frame);
  for (int i = 0; i < n; ++i) {
    const Shape& s = sh[i];
    const int cx = s.cx + ox - (view ? s.disp : 0);
    const int cy = s.cy;
    int y0 = cy - s.hh, y1 = cy + s.hh, x0 = cx - s.hw, x1 = cx + s.hw;
    if (y0 < 0) y0 = 0;
    if (x0 < 0) x0 = 0;
    if (y1 > H - 1) y1 = H - 1;
    if (x1 > W - 1) x1 = W - 1;
    const long a2 = (long)s.hw * s.hw, b2 = (long)s.hh * s.hh;
    for (int y = y0; y <= y1; ++y) {
      const long dy = y - cy;
      for (int x = x0; x <= x1; ++x) {
        if (s.kind) {
          const long dx = x - cx;
          if (dx * dx * b2 + dy * dy * a2 > a2 * b2) continue;
        }
        buf[(size_t)y * W + x] = s.val;
      }
    }
  }

  const uint64_t nseed = mix64(seed ^ ((uint64_t)frame << 20) ^ ((uint64_t)view << 52));
  for (int y = 0; y < H; ++y) {
    uint8_t* row = out + (size_t)y * stride;
    for (int x = 0; x < W; ++x) {
      int v = buf[(size_t)y * W + x] +
              (int)(mix64(nseed + (uint64_t)y * 0x100000001ull + (uint64_t)x) % 9) - 4;
      row[x] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
    }
  }
  delete[] buf;
  delete[] sh;
}

// 70 % of map points copy a frame keypoint (proj jittered by
// U(-1,1), level +U{0,1}, descriptor with ~8 % bit flips), 30 % random.
static inline void local_map(uint64_t seed, const orb_keypoint_t* keys, const uint8_t* desc,
                             int n_kp, int n_mp, int W, int H, orb_mp_track_t* mps,
                             uint8_t* mp_desc, uint8_t* kp_locked) {
  Rng r(seed * 0x9E3779B97F4A7C15ull + 0x4D415053ull);
  for (int i = 0; i < n_mp; ++i) {
    orb_mp_track_t& m = mps[i];
    uint8_t* d = mp_desc + (size_t)i * 32;
    if (n_kp > 0 && r.below(100) < 70) {
      const int k = (int)r.below((uint32_t)n_kp);
      m.proj_x = keys[k].x + (float)((int)r.below(2001) - 1000) / 1000.0f;
      m.proj_y = keys[k].y + (float)((int)r.below(2001) - 1000) / 1000.0f;
      int lvl = keys[k].octave + (int)r.below(2);
      m.level = lvl > 7 ? 7 : lvl;
      memcpy(d, desc + (size_t)k * 32, 32);
      for (int b = 0; b < 256; ++b)
        if (r.below(100) < 8) d[b >> 3] ^= (uint8_t)(1u << (b & 7));
    } else {
      m.proj_x = (float)r.below((uint32_t)W * 16u) / 16.0f;
      m.proj_y = (float)r.below((uint32_t)H * 16u) / 16.0f;
      m.level = (int)r.below(8);
      for (int b = 0; b < 32; ++b) d[b] = (uint8_t)r.below(256);
    }
    m.proj_xr = -1.0f;
    m.view_cos = (r.next() & 1) ? 0.999f : 0.9f;
    m.in_view = r.below(100) < 95 ? 1 : 0;
    m.bad = 0;
    m.has_obs = 1;
    m._pad = 0;
  }
  for (int k = 0; k < n_kp; ++k) kp_locked[k] = r.below(100) < 20 ? 1 : 0;
}

}  // namespace orb_synth
