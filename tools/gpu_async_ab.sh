#!/bin/bash
# GPU-box side: async texel update (bench --async-texture) with capped Adam grids (GSTEX_TEX_ADAM_GRID, 0 = full)
# vs the compute-stream update S (bench train step only), interleaved.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/async; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_trainer_sync.py tests/test_gpu_parity.py -x -q -k "adam or async or synced" --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 \
  || { echo "tests FAILED"; tail -30 $OUT/tests.log; exit 1; }
grep -E "passed|failed" $OUT/tests.log | tail -1
for rep in 1 2; do
  for g in 0 256 S; do
    if [ "$g" = "S" ]; then flag=""; env_=""; else flag="--async-texture"; env_="GSTEX_TEX_ADAM_GRID=$g"; fi
    env $env_ timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-sub $flag > $OUT/c_${g}_$rep.log 2>&1 || { echo "bench $g FAILED"; tail -20 $OUT/c_${g}_$rep.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/c_${g}_$rep.log').read().strip().splitlines()[-1]); print('$g', d['ms_per_step'], d['ms_per_step_median'])"
  done
done
