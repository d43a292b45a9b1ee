#!/bin/bash
# GPU box: the hipGraph step (gstex_amd.graphs.StepGraphs) -- its tests, then the bench with and without it and at
# the driver's --steps 20 --warmup 5.  Results under gpurun_out/graph/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/graph; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_graphs.py -x -v -s --timeout 300 --timeout-method thread \
  > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
for v in "first:" "all:--graph all" "eager:--graph none" "driver_first:--steps 20 --warmup 5" \
         "driver_all:--steps 20 --warmup 5 --graph all" "driver_eager:--steps 20 --warmup 5 --graph none"; do
  name=${v%%:*}; flags=${v#*:}
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-sub $flags > $OUT/bench_$name.log 2>&1 \
    || { tail -30 $OUT/bench_$name.log; exit 1; }
  grep '^{' $OUT/bench_$name.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.readline())
ev = d['step_ms_events']
import statistics as st
t = ev[len(ev) // 2:]
print('$name', d['ms_per_step'], 'median', d['ms_per_step_median'], 'first', ev[0], 'tail mean %.4f' % st.mean(t),
      'host', d['host_enqueue_ms_median'], 'bwd', d['kernel_ms'].get('raster_bwd'),
      d.get('config', {}).get('step_launch', '')[:30])"
done
