#!/bin/bash
# GPU-box check used during development: raster-only cfg3 timing of the working tree (and of scratch/head,
# the committed HEAD built by `git archive`, when present), then the -m gpu test suite.
#   gpurun -- bash tools/gpu_check.sh [pytest -k expression]
# VARIANTS="a b": also time scratch/<a>/libgstex_hip.so ... (tools/build_variant.sh); NOTESTS=1: timing only.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/check; mkdir -p $OUT
[ -z "$NOLOOP" ] && { timeout -k 10 180 python3 -u tools/raster_loop.py --photometric --iters 20 > $OUT/loop_new.log 2>&1 || { echo "loop_new FAILED"; tail -20 $OUT/loop_new.log; exit 1; }
echo "new : $(tail -1 $OUT/loop_new.log)"; }
if [ -d scratch/head ]; then
  (cd scratch/head && timeout -k 10 180 python3 -u tools/raster_loop.py --photometric --iters 20) > $OUT/loop_head.log 2>&1 || { echo "loop_head FAILED"; tail -5 $OUT/loop_head.log; exit 1; }
  echo "head: $(tail -1 $OUT/loop_head.log)"
fi
for rep in $(seq 1 ${REPEAT:-1}); do
for v in $VARIANTS; do
  GSTEX_LIB=scratch/$v/libgstex_hip.so timeout -k 10 180 python3 -u tools/raster_loop.py --photometric --iters ${ITERS:-20} > $OUT/loop_$v.log 2>&1 || { echo "loop_$v FAILED"; tail -5 $OUT/loop_$v.log; exit 1; }
  echo "$v: $(tail -1 $OUT/loop_$v.log)"
done
done
[ -n "$NOTESTS" ] && exit 0
K=${1:-}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread ${K:+-k "$K"} > $OUT/gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed|error" $OUT/gpu_tests.log | tail -3
exit $rc
