#!/bin/bash
# The committed HEAD as a whole tree in scratch/head (sources + its own python + built library): tools/gpu_check.sh
# times it beside the working tree (A/B across ABI changes, since each tree loads its own library).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
rm -rf "$ROOT/scratch/head"
mkdir -p "$ROOT/scratch/head"
cd "$ROOT"
git archive HEAD | tar -x -C scratch/head
make -s -C scratch/head/gstex_amd/csrc -j8
echo "built scratch/head (HEAD $(git rev-parse --short HEAD))"
