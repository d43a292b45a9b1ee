#!/bin/bash
# Builds an experimental variant of libgstex_hip.so with extra -D flags, for A/B timing on the GPU box:
#   tools/build_variant.sh NAME -DGSTEX_ABLATE=1 ...   -> scratch/NAME/libgstex_hip.so
# Run it with GSTEX_LIB=scratch/NAME/libgstex_hip.so python tools/raster_loop.py ...
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/scratch/$NAME"
make -s -C "$ROOT/gstex_amd/csrc" -j8 OBJDIR="$ROOT/scratch/$NAME/obj" OUT="$ROOT/scratch/$NAME/libgstex_hip.so" EXTRA="$*"
echo "built scratch/$NAME ($*)"
