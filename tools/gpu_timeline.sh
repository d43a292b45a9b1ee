#!/bin/bash
# GPU-box side: per-wave backward timeline (GSTEX_STATS=3 builds, tools/build_variant.sh NAME -DGSTEX_STATS=3 ...)
# for each scratch/<NAME> given, summarised by tools/wg_timeline.py.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/tl
for v in "$@"; do
  GSTEX_LIB=scratch/$v/libgstex_hip.so GSTEX_WG_DUMP=gpurun_out/tl/$v.npy timeout -k 10 120 python3 tools/raster_loop.py --photometric --iters 10 > gpurun_out/tl/$v.log 2>&1 || { echo "FAIL $v"; exit 1; }
  echo "== $v: $(grep -o "raster_bwd': [0-9.]*" gpurun_out/tl/$v.log)"
  python3 tools/wg_timeline.py gpurun_out/tl/$v.npy 65536 | head -3
done
