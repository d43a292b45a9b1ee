#!/bin/bash
# GPU tests + raster A/B vs HEAD, then the bench line and the rocprofv3 passes.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_check.sh || exit 1
bash tools/gpu_r03_bench.sh
