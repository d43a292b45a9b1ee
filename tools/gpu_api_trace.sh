#!/bin/bash
# HIP API + memory-copy + kernel trace of a short bench run (no PMC counters): which calls a training step makes
# (memsets, copies and their directions, synchronisations).  Output: gpurun_out/api_<TAG>/
TAG=${1:-cur}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/api_$TAG; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --hip-trace --memory-copy-trace --kernel-trace --output-format csv -d $OUT -o run -- \
  python3 bench.py --steps 6 --warmup 3 --no-sub --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
ls $OUT
