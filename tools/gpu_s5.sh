#!/bin/bash
# -m gpu suite on the tree's library, then raster-loop A/B of scratch variants (args).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/s5; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
tail -3 $OUT/gpu_tests.log
[ $rc = 0 ] || exit $rc
FILTER="raster_bwd|raster_fwd" timeout -k 10 500 bash tools/gpu_trace_variants.sh "$@" && \
FILTER="raster_bwd|raster_fwd" timeout -k 10 500 bash tools/gpu_trace_variants.sh "$@"
