#!/bin/bash
# Session check: -m gpu suite + default bench line + the quadrant-pair visit census.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/s1; mkdir -p $OUT
timeout -k 10 120 python3 -u tools/pair_union.py > $OUT/pair_union.log 2>&1 || { echo "pair_union FAILED"; tail -20 $OUT/pair_union.log; exit 1; }
cat $OUT/pair_union.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed|error" $OUT/gpu_tests.log | tail -3
[ $rc = 0 ] || exit $rc
timeout -k 10 500 python3 -u bench.py > $OUT/bench.log 2>&1 || { echo "bench FAILED"; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-400
