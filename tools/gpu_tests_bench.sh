#!/bin/bash
# GPU-box side: the -m gpu suite, then the default bench line (no profile).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/check; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed|error" $OUT/gpu_tests.log | tail -3
[ $rc = 0 ] || exit $rc
timeout -k 10 500 python3 -u bench.py > $OUT/bench.log 2>&1 || { echo "bench FAILED"; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-330
if [ -d scratch/head ]; then
  (cd scratch/head && timeout -k 10 500 python3 -u bench.py --no-sub --no-cpu-baseline) > $OUT/bench_head.log 2>&1 || { echo "head bench FAILED"; exit 1; }
  echo "head: $(tail -1 $OUT/bench_head.log | cut -c1-330)"
fi
