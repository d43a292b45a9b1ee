#!/bin/bash
# Interleaved bench A/B over environment settings of the same tree: each argument is one variant's env assignment
# list (e.g. "GSTEX_DEFER_SIDE=0" "GSTEX_DEFER_SIDE=1"); the timed train step only.  SKIP_TESTS unset: -m gpu first.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/envab; mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/gpu_tests.log 2>&1
  rc=$?
  tail -2 $OUT/gpu_tests.log
  [ $rc = 0 ] || exit $rc
fi
for rep in 1 2 3; do
  i=0
  for v in "$@"; do
    i=$((i+1))
    ( export $v; timeout -k 10 300 python3 -u bench.py --no-sub --no-cpu-baseline --steps ${STEPS:-60} ) > $OUT/bench_${i}_$rep.log 2>&1 || { echo "bench [$v] FAILED"; tail -5 $OUT/bench_${i}_$rep.log; exit 1; }
    python3 - "$OUT/bench_${i}_$rep.log" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ev = sorted(d.get('step_ms_events', []))
spk = [round(x, 2) for x in d.get('step_ms_events', []) if x > 2.6]
print(f"{sys.argv[2]:24s} mean {d['ms_per_step']:.4f} median {d['ms_per_step_median']:.4f} ms  kernels {d.get('kernel_ms')} spikes>2.6 {spk}")
PY
  done
done
