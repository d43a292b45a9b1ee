#!/bin/bash
# gstex_amd.fused A/B (gpurun -- bash tools/gpu_fused_ab.sh TAG): its GPU tests, the host time to the raster forward
# per path (tools/host_breakdown.py), and the driver's bench command alternating GSTEX_FUSED_STEP=0/1 (ROUNDS pairs).
TAG=${1:?usage: gpu_fused_ab.sh TAG}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fused.py -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
  tail -1 $OUT/tests.log
fi
for f in 0 1; do
  GSTEX_FUSED_STEP=$f timeout -k 10 240 python3 -u tools/host_breakdown.py > $OUT/host_$f.log 2>&1 || { tail -20 $OUT/host_$f.log; exit 1; }
  echo "fused=$f"; head -3 $OUT/host_$f.log
done
for r in $(seq 1 ${ROUNDS:-2}); do
  for f in 0 1; do
    GSTEX_FUSED_STEP=$f timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $OUT/bench_${f}_$r.log 2>&1 || { tail -20 $OUT/bench_${f}_$r.log; exit 1; }
    python3 - $OUT/bench_${f}_$r.log $f <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s = d["step_ms_events"]
print(f"fused={sys.argv[2]} mean {d['ms_per_step']:.4f} median {d['ms_per_step_median']:.4f} first {s[0]:.3f} "
      f"fwd {d['roofline'].get('achieved')}")
PY
  done
done
