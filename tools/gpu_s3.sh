#!/bin/bash
# Round-3 evidence at HEAD: -m gpu suite, the default bench line, rocprofv3 trace + PMC passes (profiles/).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/s3; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed|error" $OUT/gpu_tests.log | tail -3
[ $rc = 0 ] || exit $rc
timeout -k 10 500 python3 -u bench.py > $OUT/bench.log 2>&1 || { echo "bench FAILED"; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-400
timeout -k 10 1200 bash tools/profile_bench.sh ${TAG:-r03s} > $OUT/prof.log 2>&1 || { echo "profile FAILED"; tail -20 $OUT/prof.log; exit 1; }
echo profile done
