#!/bin/bash
# GPU-box side: the raster parity tests against an experimental library build (tools/build_variant.sh NAME ...):
#   gpurun -- bash tools/gpu_variant_tests.sh NAME [pytest -k expression]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/check; mkdir -p $OUT
V=$1; K=${2:-}
GSTEX_LIB=scratch/$V/libgstex_hip.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_deep.py \
  -m gpu -x -q --timeout 150 --timeout-method thread ${K:+-k "$K"} > $OUT/variant_tests_$V.log 2>&1
rc=$?
grep -E "passed|failed|error" $OUT/variant_tests_$V.log | tail -3
exit $rc
