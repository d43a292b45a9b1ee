#!/bin/bash
# Round-3 measurement: the default bench line, then the rocprofv3 trace + PMC passes of the timed loop (profiles/).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r03; mkdir -p $OUT
timeout -k 10 500 python3 -u bench.py > $OUT/bench.log 2>&1 || { echo "bench FAILED"; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-400
timeout -k 10 1200 bash tools/profile_bench.sh ${TAG:-r03} > $OUT/prof.log 2>&1 || { echo "profile FAILED"; tail -20 $OUT/prof.log; exit 1; }
echo profile done
