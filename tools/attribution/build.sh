#!/bin/bash
# Build an attribution / A-B variant of liborb_amd.so that the product source
# no longer carries:
#   tools/attribution/build.sh NAME "-DFC_STUB=2"
# -> orb_slam2-chinese-annotation_amd/lib/variants/NAME.so, built from a copy of
# the product csrc/ with variants.patch applied, which restores:
#   FC_STUB=1..5      k_fast_cells phase stubs (results wrong)
#   FC_STAMPS         k_fast_cells per-phase s_memtime stamps (tools/probe/fc_stamps.py)
#   ORB_FAST_STAMPS   k_fast_band per-phase stamps
#   DESC_STUB=1..5    k_orient_desc phase stubs (results wrong)
#   DESC_GLDS, DESC_LDS_PAD, DESC_DBUF, DESC_MFMA_ROWS, DESC_PK_ROT,
#   FC_LDS_PAD_TILES  measured-slower k_orient_desc / k_fast_cells variants
# PATCHES=fast_runs.patch instead restores k_fast_runs (round 6: FAST over runs
# of ORB_FAST_RUN_CELLS cells per wave; measured slower).
# Select the build with ORB_AMD_LIB=<path>.  variants.patch is the diff from
# the product file to the round-5 source that held these blocks inline
# (regenerate: tools/unifdef.py resolves them, see its docstring).
set -e
NAME=$1; FLAGS=$2
R=$(cd "$(dirname "$0")/../.." && pwd)
PKG="$R/orb_slam2-chinese-annotation_amd"
W=$(mktemp -d)
trap 'rm -rf "$W"' EXIT
mkdir -p "$W/pkg"
cp -r "$PKG/csrc" "$W/pkg/csrc"
cp "$PKG/Makefile" "$W/pkg/Makefile"
ln -s "$R/include" "$W/include"
for p in ${PATCHES:-variants.patch}; do  # e.g. PATCHES=fast_runs.patch
  patch -s -d "$W/pkg" -p1 < "$R/tools/attribution/$p"
done
make -s -j8 -C "$W/pkg" BUILD=build LIBOUT="$PKG/lib/variants/$NAME.so" EXTRA_HIPFLAGS="$FLAGS"
echo "$PKG/lib/variants/$NAME.so"
