#!/bin/bash
# The -m gpu suite, then the fused-prologue A/B (tools/gpu_fused_ab.sh TAG without its test step) and a kernel trace of
# the driver's bench command summarised per kernel (gpurun -- bash tools/gpu_fused_round.sh TAG).
TAG=${1:?usage: gpu_fused_round.sh TAG}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { grep -E "FAIL|Error|error" $OUT/gpu_tests.log | head -20; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
if [ -z "$SKIP_AB" ]; then SKIP_TESTS=1 ROUNDS=${ROUNDS:-2} bash tools/gpu_fused_ab.sh $TAG || exit 1; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --no-sub --no-cpu-baseline --steps 20 --warmup 5 > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
python3 tools/first_step_trace.py $OUT/trace/run_kernel_trace.csv 5 > $OUT/first_step.txt && head -22 $OUT/first_step.txt
