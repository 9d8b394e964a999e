#!/bin/bash
# Build an alternate liborb_amd.so with extra compile flags for A/B runs:
#   tools/build_variant.sh NAME "-DFC_WAVES=1 -DFC_CPW=8"
# -> orb_slam2-chinese-annotation_amd/lib/variants/NAME.so; select it with
#    ORB_AMD_LIB=orb_slam2-chinese-annotation_amd/lib/variants/NAME.so
set -e
NAME=$1; FLAGS=$2
D=$(cd "$(dirname "$0")/../orb_slam2-chinese-annotation_amd" && pwd)
make -s -j8 -C "$D" BUILD=build_var/$NAME LIBOUT=lib/variants/$NAME.so EXTRA_HIPFLAGS="$FLAGS"
