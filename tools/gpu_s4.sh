#!/bin/bash
# A/B of backward variants (raster loop under rocprofv3), two interleaved passes.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
FILTER="raster_bwd|raster_fwd" timeout -k 10 500 bash tools/gpu_trace_variants.sh "$@" && \
FILTER="raster_bwd" timeout -k 10 500 bash tools/gpu_trace_variants.sh "$@"
