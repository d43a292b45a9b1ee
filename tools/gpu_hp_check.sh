#!/bin/bash
# GPU-box side (gpurun -- bash tools/gpu_hp_check.sh TAG): the raster parity / deep-window tests (their printed
# per-gradient errors vs the fp64 oracle), then the cfg3 raster loop with the near-edge-on fp64 path off / on
# (GSTEX_HP=0 / 1), interleaved, for its cost.
TAG=${1:-hp}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_deep.py tests/test_gpu_parity.py -k "raster or cfg" -v -s \
  --timeout 300 --timeout-method thread > $OUT/parity.log 2>&1; echo "parity rc $?"
grep -E "passed|failed" $OUT/parity.log | tail -1
for i in 1 2; do
  for hp in 0 1; do
    GSTEX_HP=$hp timeout -k 10 120 python3 tools/raster_loop.py --photometric --no-geometry --iters 20 > $OUT/loop_hp${hp}_$i.log 2>&1 || { echo "loop failed"; exit 1; }
    echo "hp=$hp #$i: $(tail -2 $OUT/loop_hp${hp}_$i.log | tr '\n' ' ')"
  done
done
