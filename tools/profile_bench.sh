#!/bin/bash
# Collects the round's rocprofv3 evidence on the GPU box (run via gpurun from the repo root):
#   1. --kernel-trace --stats of the default bench command (timing; agrees with bench.py's events)
#   2. --pmc FETCH_SIZE and 3. --pmc WRITE_SIZE in separate passes (TCC slots: 3 + 2 > 4)
#   4. --pmc SQ_INSTS_VALU SQ_WAVES (wave-level VALU instructions per launch: the issue roofline)
# Output: gpurun_out/prof_<tag>/...; summarise locally with tools/summarize_profiles.py <tag>.
set -e
TAG=${1:-r03}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
# same step/warmup counts as the default bench line, so the steady-state averages agree
BENCH="python3 bench.py --no-cpu-baseline --no-sub"  # the timed train-step loop only
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- $BENCH > "$OUT/bench_trace.log" 2>&1
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- $BENCH > "$OUT/bench_fetch.log" 2>&1
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- $BENCH > "$OUT/bench_write.log" 2>&1
timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --output-format csv -d "$OUT/valu" -o run -- $BENCH > "$OUT/bench_valu.log" 2>&1
echo done
