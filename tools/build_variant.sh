#!/bin/bash
# Builds an experimental variant of libgstex_hip.so with extra -D flags, for A/B timing on the GPU box:
#   tools/build_variant.sh NAME -DGSTEX_ABLATE=1 ...   -> scratch/NAME/libgstex_hip.so
#   PATCH=tools/variants/bwd_merge.patch tools/build_variant.sh NAME -DGSTEX_BWD_MERGE=1
#     (an experiment kept out of the product sources: the patch is applied to a copy of gstex_amd/csrc)
# Run it with GSTEX_LIB=scratch/NAME/libgstex_hip.so python tools/raster_loop.py ...
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/scratch/$NAME"
SRC="$ROOT/gstex_amd/csrc"
if [ -n "$PATCH" ]; then
  # the copy keeps the tree shape the Makefile's relative include path expects (csrc/../../include)
  rm -rf "$ROOT/scratch/$NAME/src" "$ROOT/scratch/$NAME/include"
  mkdir -p "$ROOT/scratch/$NAME/src/csrc" && cp -r "$ROOT/include" "$ROOT/scratch/$NAME/include"
  cp "$SRC"/Makefile "$SRC"/*.hip "$SRC"/*.h "$ROOT/scratch/$NAME/src/csrc/"
  patch -s -p1 -d "$ROOT/scratch/$NAME/src/csrc" < "$ROOT/$PATCH"
  SRC="$ROOT/scratch/$NAME/src/csrc"
fi
make -s -C "$SRC" -j8 OBJDIR="$ROOT/scratch/$NAME/obj" OUT="$ROOT/scratch/$NAME/libgstex_hip.so" EXTRA="$*"
echo "built scratch/$NAME ($*${PATCH:+, $PATCH})"
