#!/bin/bash
# The first timed step (gpurun -- bash tools/gpu_first_step.sh TAG): host time to each entry point of an eager step
# started after a synchronisation (tools/host_breakdown.py), the driver's bench command twice and the default bench
# once (their first step against the median), and a kernel trace of the driver's command analysed by
# tools/first_step_trace.py (the first timed step's kernels and idle gaps against the steady steps).
TAG=${1:?usage: gpu_first_step.sh TAG}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 240 python3 -u tools/host_breakdown.py > $OUT/host.log 2>&1 || { tail -20 $OUT/host.log; exit 1; }
grep -v amdgpu.ids $OUT/host.log | head -12
summ() {
python3 - "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s = d["step_ms_events"]
print(f"{sys.argv[1]}: mean {d['ms_per_step']:.4f} median {d['ms_per_step_median']:.4f} first {s[0]:.3f} "
      f"({100 * (s[0] / d['ms_per_step_median'] - 1):.1f} %) gap {100 * (d['ms_per_step'] / d['ms_per_step_median'] - 1):.2f} %")
PY
}
for r in 1 2; do
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $OUT/driver_$r.log 2>&1 || { tail -20 $OUT/driver_$r.log; exit 1; }
  summ $OUT/driver_$r.log
done
timeout -k 10 400 python3 -u bench.py > $OUT/default.log 2>&1 || { tail -20 $OUT/default.log; exit 1; }
summ $OUT/default.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 bench.py --no-sub --no-cpu-baseline --steps 20 --warmup 5 > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
python3 tools/first_step_trace.py $OUT/trace/run_kernel_trace.csv 5 > $OUT/first_step.txt && head -3 $OUT/first_step.txt && tail -1 $OUT/first_step.txt
