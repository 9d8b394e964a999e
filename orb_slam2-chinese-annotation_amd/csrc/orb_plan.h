// orb_plan.h -- per-image-size extraction plan shared by the host runtime and kernels.
//
// Everything that depends only on (width, height, nfeatures, scaleFactor,
// nlevels) is computed once on the host -- level sizes, resize coefficient
// tables, the FAST cell grid, octree root layout, output slot layout -- with
// the exact float/double expressions of the reference
// (src/ORBextractor.cc:428-489, 785-815, 558-582, 1172-1207), and handed to
// the kernels by value.  The kernels then do only per-pixel / per-key work.
#pragma once
#include <stdint.h>

#ifndef ORB_MAX_LEVELS
#define ORB_MAX_LEVELS 16
#endif

struct OrbLevelDesc {
  int w, h;          // level size (cvRound(W * invScale), src/ORBextractor.cc:1180)
  int pitch;         // row pitch of the level in the pyramid arena (level 0: caller stride)
  int blurPitch;     // row pitch of the level's blurred copy
  long long arenaOff;// byte offset of the level inside one image's pyramid arena (l >= 1)
  long long blurOff; // byte offset of the blurred level inside one image's blur arena
  int cellBeg, cellEnd;  // range of this level's cells in the cell table
  int quota;         // mnFeaturesPerLevel[l]
  int nodeCap;       // max alive octree nodes == max keypoints this level can emit
  int outOff;        // first output slot of this level inside one image's slot arena
  int nIni;          // octree root count (src/ORBextractor.cc:562)
  float hX;          // root width (src/ORBextractor.cc:564)
  int Wr, Hr;        // maxBorderX-minBorderX, maxBorderY-minBorderY
  float scale;       // mvScaleFactor[l]
  float sizeF;       // (float)(int)(31 * scale), src/ORBextractor.cc:874
  int rtabX, rtabY;  // offsets of this level's resize tables (x: xofs/alpha, y: yofs/beta)
  int xmax;          // first dx whose source tap sx+1 falls outside (resize)
  int resizeMode;    // ORB_RESIZE_NARROW / _WIDE / _GENERIC: k_pyr_resize variant for this level
  int tileBeg;       // first blur tile of this level
  int cellMaxRows, cellMaxCols;  // largest cell ROI of this level (k_fast_cells LDS per launch)
  int resize2;       // 1: levels l and l + 1 are built by one k_pyr_resize2 launch (from l - 1)
};

#define ORB_RESIZE_NARROW 0   // 44 x 44-dword source windows (downscale <= 1.25)
#define ORB_RESIZE_WIDE 1     // 64 x 64 dwords
#define ORB_RESIZE_GENERIC 2  // untiled: each thread reads its taps from the source level

struct OrbPlanDesc {
  int nlevels;
  int ncells;        // total FAST cells over all levels
  int keyCap;        // per-cell candidate capacity (max strict NMS maxima in a cell window)
  int slotsPerImage; // sum of nodeCap over levels
  int iniTh, minTh;
  int maxCellRows, maxCellCols;  // largest cell ROI (for LDS sizing)
  int srcW, srcH;
  int nBlurTiles;    // blur tiles over all levels of one image
  int nBands;        // FAST bands over all levels
  int maxBandBytes;  // largest FAST band in elements: rows x LDS pitch ((cols + 20) & ~7)
  OrbLevelDesc lv[ORB_MAX_LEVELS];
};

// One FAST cell: ROI rows [y0,y1) x cols [x0,x1) of its level image
// (src/ORBextractor.cc:816-839).  Cells are ordered level-major, then
// row-major, i.e. the order in which the reference appends to vToDistributeKeys.
struct OrbCellDesc {
  int16_t level, y0, y1, x0, x1, _pad;
};

// One FAST band: cells [cellBeg, cellBeg + nCells) of one cell row of one
// level (consecutive in the cell table); rows [y0,y1) x cols [x0,x1) is the
// union of their ROIs.
struct OrbBandDesc {
  int16_t level, y0, y1, x0, x1, nCells;
  int32_t cellBeg;
};
#ifndef ORB_OCTREE_LDS_KB
#define ORB_OCTREE_LDS_KB 52  // k_octree node tables + keys per workgroup (swept 24-64)
#endif
#define ORB_BAND_BYTES 6656  // elements (rows x LDS pitch) of one FAST band: f16 pixels + strengths; 5 workgroups per CU (swept 4-10 K)

// One ORB_BLUR_TW x ORB_BLUR_TH output tile of the 7x7 Gaussian pass over level `level`.
struct OrbTileDesc {
  int16_t level, x0, y0, _pad;
};
#define ORB_BLUR_TW 128
#define ORB_BLUR_TH 32

