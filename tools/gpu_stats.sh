#!/bin/bash
# GPU-box side: work counters of a GSTEX_STATS=1 build (tools/build_variant.sh stats -DGSTEX_STATS=1) over the cfg3
# photometric raster loop: backward visits / lanes / flushes and the forward's cull yield.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/check
GSTEX_LIB=scratch/stats/libgstex_hip.so timeout -k 10 180 python3 -u tools/raster_loop.py --photometric --iters 5 \
  > gpurun_out/check/stats.log 2>&1 || { echo "stats FAILED"; tail -5 gpurun_out/check/stats.log; exit 1; }
grep "stats/launch" gpurun_out/check/stats.log
