#!/bin/bash
# -m gpu suite on the tree's library, then interleaved bench A/B: the tree's library vs scratch/<variant> libraries
# (python side shared; GSTEX_LIB selects the library), the timed train step only.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/ab; mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/gpu_tests.log 2>&1
  rc=$?
  tail -2 $OUT/gpu_tests.log
  [ $rc = 0 ] || exit $rc
fi
for rep in 1 2; do
  for v in tree "$@"; do
    if [ "$v" = tree ]; then lib=gstex_amd/libgstex_hip.so; else lib=scratch/$v/libgstex_hip.so; fi
    GSTEX_LIB=$lib timeout -k 10 300 python3 -u bench.py --no-sub --no-cpu-baseline --steps 40 > $OUT/bench_${v}_$rep.log 2>&1 || { echo "bench $v FAILED"; tail -5 $OUT/bench_${v}_$rep.log; exit 1; }
    python3 - "$OUT/bench_${v}_$rep.log" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:10s} mean {d['ms_per_step']:.4f} median {d['ms_per_step_median']:.4f} ms  kernels {d.get('kernel_ms')}")
PY
  done
done
