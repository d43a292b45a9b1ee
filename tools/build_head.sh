#!/bin/bash
# Builds the library from the committed HEAD sources into scratch/prev/ (A/B baseline for tools/gpu_ablate.sh).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
rm -rf "$ROOT/scratch/prev_csrc" "$ROOT/scratch/prev"
mkdir -p "$ROOT/scratch/prev_csrc"
cd "$ROOT"
for f in $(git ls-files gstex_amd/csrc); do git show HEAD:$f > scratch/prev_csrc/$(basename $f); done
make -s -C scratch/prev_csrc -j8 OBJDIR="$ROOT/scratch/prev/obj" OUT="$ROOT/scratch/prev/libgstex_hip.so"
echo "built scratch/prev (HEAD)"
