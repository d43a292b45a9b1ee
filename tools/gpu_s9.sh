#!/bin/bash
# -m gpu suite, then the bench line twice and a kernel trace of the train step (Adam, raster fwd, fills).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/s9; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -1 $OUT/gpu_tests.log
[ $rc = 0 ] || { grep -E "Error|assert" $OUT/gpu_tests.log | head -20; exit $rc; }
for i in 1 2; do
  timeout -k 10 300 python3 -u bench.py --no-sub --no-cpu-baseline > $OUT/bench_$i.log 2>&1 || { echo "bench FAILED"; tail -5 $OUT/bench_$i.log; exit 1; }
  tail -1 $OUT/bench_$i.log | cut -c1-220
done
FILTER="adam|raster_fwd|Fill|fill" timeout -k 10 300 bash tools/gpu_trace_bench.sh
