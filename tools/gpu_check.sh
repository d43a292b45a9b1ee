#!/bin/bash
# GPU-box check used during development: raster-only cfg3 timing of the working tree's library and of
# scratch/<variant> libraries (tools/build_variant.sh), then a subset of the -m gpu test suite.
#   gpurun -- 'VARIANTS="a b" REPEAT=2 bash tools/gpu_check.sh [pytest -k expression]'
# NOLOOP=1: no timing; NOTESTS=1: timing only.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/check; mkdir -p $OUT
if [ -z "$NOLOOP" ]; then
  for rep in $(seq 1 ${REPEAT:-1}); do
    for v in tree $VARIANTS; do
      if [ "$v" = tree ]; then lib=gstex_amd/libgstex_hip.so; else lib=scratch/$v/libgstex_hip.so; fi
      GSTEX_LIB=$lib timeout -k 10 180 python3 -u tools/raster_loop.py --photometric --iters ${ITERS:-20} > $OUT/loop_$v.log 2>&1 || { echo "loop $v FAILED"; tail -5 $OUT/loop_$v.log; exit 1; }
      echo "$v: $(tail -1 $OUT/loop_$v.log)"
    done
  done
fi
[ -n "$NOTESTS" ] && exit 0
K=${1:-}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${K:+-k "$K"} > $OUT/gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed|error" $OUT/gpu_tests.log | tail -3
exit $rc
