#!/bin/bash
# A/B raster timing (working tree vs scratch/prev = HEAD build), backward work counters (scratch/stats), deep parity report.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r03; mkdir -p $OUT
VARIANTS="${VARIANTS:-prev}" NOTESTS=1 REPEAT=${REPEAT:-2} bash tools/gpu_check.sh || exit 1
if [ -f scratch/stats/libgstex_hip.so ]; then bash tools/gpu_stats.sh || exit 1; fi
[ -n "$NODEEP" ] && exit 0
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_deep.py tests/test_conventions.py -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/deep_parity.log 2>&1
rc=$?; grep -E "passed|failed" $OUT/deep_parity.log | tail -2; exit $rc
