#!/bin/bash
# A round's GPU evidence in one call (gpurun -- bash tools/gpu_round.sh TAG): the -m gpu suite, smoke(), the default
# bench line, the driver's bench command (--steps 20 --warmup 5), and the rocprofv3 trace + PMC passes of the bench
# (tools/profile_bench.sh TAG).  Outputs under gpurun_out/TAG/ and gpurun_out/prof_TAG/; summarise locally with
# tools/summarize_profiles.py TAG.  SKIP_TESTS=1 / SKIP_PROF=1 skip those parts.
TAG=${1:?usage: gpu_round.sh TAG}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
  grep -E "passed|failed" $OUT/gpu_tests.log | tail -1
  timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
timeout -k 10 400 python3 -u bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-300
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $OUT/bench_driver_cmd.log 2>&1 || { tail -20 $OUT/bench_driver_cmd.log; exit 1; }
tail -1 $OUT/bench_driver_cmd.log | cut -c1-200
if [ -z "$SKIP_PROF" ]; then
  timeout -k 10 1200 bash tools/profile_bench.sh $TAG > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
  tail -2 $OUT/prof.log
fi
