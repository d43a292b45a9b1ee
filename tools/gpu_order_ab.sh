#!/bin/bash
# GSTEX_ORDER_AHEAD A/B (gpurun -- bash tools/gpu_order_ab.sh TAG): its GPU test, then the driver's bench command
# alternating GSTEX_ORDER_AHEAD=0/1 (ROUNDS pairs) and a kernel trace with it on.
TAG=${1:?usage: gpu_order_ab.sh TAG}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fused.py -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in $(seq 1 ${ROUNDS:-3}); do
  for f in 0 1; do
    GSTEX_ORDER_AHEAD=$f timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $OUT/bench_${f}_$r.log 2>&1 || { tail -20 $OUT/bench_${f}_$r.log; exit 1; }
    python3 - $OUT/bench_${f}_$r.log $f <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s = d["step_ms_events"]
print(f"order_ahead={sys.argv[2]} mean {d['ms_per_step']:.4f} median {d['ms_per_step_median']:.4f} first {s[0]:.3f}")
PY
  done
done
GSTEX_ORDER_AHEAD=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 bench.py --no-sub --no-cpu-baseline --steps 20 --warmup 5 > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
python3 tools/first_step_trace.py $OUT/trace/run_kernel_trace.csv 5 > $OUT/first_step.txt && head -2 $OUT/first_step.txt
