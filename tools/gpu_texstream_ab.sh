#!/bin/bash
# A/B of the side-stream texel update (GStexTrainer texture_stream, GSTEX_TEX_STREAM / GSTEX_TEX_GRID) on the bench:
# interleaved runs at the driver's settings; one line per run (mean, median, first step, tail mean).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/texstream; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_trainer_sync.py -x -q --timeout 200 --timeout-method thread \
  -k texture_stream > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for rep in 1 2; do
  for v in "base:0:0" "side0:1:0" "side256:1:256" "side128:1:128" "side64:1:64"; do
    IFS=: read name ts grid <<< "$v"
    GSTEX_TEX_STREAM=$ts GSTEX_TEX_GRID=$grid timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline \
      --no-sub > $OUT/${name}_$rep.log 2>&1 || { tail -20 $OUT/${name}_$rep.log; exit 1; }
    grep '^{' $OUT/${name}_$rep.log | python3 -c "
import json, statistics as st, sys
d = json.loads(sys.stdin.readline()); e = d['step_ms_events']; t = e[len(e) // 2:]
print('$name', '$rep', d['ms_per_step'], 'median', d['ms_per_step_median'], 'first', e[0], 'tail %.4f' % st.mean(t),
      'bwd', d['kernel_ms'].get('raster_bwd'), 'fwd', d['kernel_ms'].get('raster_fwd'))"
  done
done
