#!/bin/bash
# Kernel trace of the driver bench command per path (GSTEX_FUSED_STEP=1/0) and the first timed step against a steady
# step (tools/first_step_trace.py).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/fst; mkdir -p $OUT
for f in 1 0; do
GSTEX_FUSED_STEP=$f timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/f$f -o run -- python3 bench.py --no-sub --no-cpu-baseline --steps 20 --warmup 5 > $OUT/f$f.log 2>&1 || { tail -20 $OUT/f$f.log; exit 1; }
python3 tools/first_step_trace.py $(ls $OUT/f$f/*/run_kernel_trace.csv $OUT/f$f/run_kernel_trace.csv 2>/dev/null | head -1) > $OUT/f$f.txt; cat $OUT/f$f.txt | head -60
done
