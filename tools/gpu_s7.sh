#!/bin/bash
# Round-3 final evidence at HEAD: -m gpu suite, smoke(), the default bench line, the driver's bench command
# (--steps 20 --warmup 5), rocprofv3 trace + PMC passes (profiles/).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/s7; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed|error" $OUT/gpu_tests.log | tail -2
[ $rc = 0 ] || exit $rc
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke FAILED"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 500 python3 -u bench.py > $OUT/bench.log 2>&1 || { echo "bench FAILED"; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-300
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.log 2>&1 || { echo "driver bench FAILED"; exit 1; }
tail -1 $OUT/bench_driver.log | cut -c1-300
timeout -k 10 1200 bash tools/profile_bench.sh ${TAG:-r03t} > $OUT/prof.log 2>&1 || { echo "profile FAILED"; tail -20 $OUT/prof.log; exit 1; }
echo profile done
