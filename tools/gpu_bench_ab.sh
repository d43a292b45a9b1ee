#!/bin/bash
# Interleaved A/B of the driver's bench command (gpurun -- bash tools/gpu_bench_ab.sh TAG "ARGS_A" "ARGS_B" [ROUNDS]):
# mean / median / first step of `bench.py --steps 20 --warmup 5 ARGS` alternating A and B.
TAG=${1:?usage: gpu_bench_ab.sh TAG ARGS_A ARGS_B [ROUNDS]}; A=$2; B=$3; R=${4:-3}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
for r in $(seq 1 $R); do
  for x in A B; do
    if [ $x = A ]; then args=$A; else args=$B; fi
    timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 $args > $OUT/bench_${x}_$r.log 2>&1 || { tail -20 $OUT/bench_${x}_$r.log; exit 1; }
    python3 - $OUT/bench_${x}_$r.log "$x: $args" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s = d["step_ms_events"]
print(f"{sys.argv[2]:40s} mean {d['ms_per_step']:.4f} median {d['ms_per_step_median']:.4f} first {s[0]:.3f} "
      f"bwd {d['roofline']['launch_ms']}")
PY
  done
done
