#!/bin/bash
# GPU-box side (gpurun -- bash tools/gpu_loop_ab.sh TAG "LABEL=ENV..." ...): the cfg3 training-path raster loop
# (tools/raster_loop.py --photometric --no-geometry) under each labelled environment (e.g. a GSTEX_LIB variant from
# tools/build_variant.sh, GSTEX_HP=0), interleaved twice, for A/B timing of the forward and backward kernels.
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
for i in 1 2; do
  for cfg in "$@"; do
    label=${cfg%%=*}; envs=${cfg#*=}
    env $envs timeout -k 10 120 python3 tools/raster_loop.py --photometric --no-geometry --iters 20 > $OUT/${label}_$i.log 2>&1 || { echo "$label failed"; tail -5 $OUT/${label}_$i.log; exit 1; }
    echo "$label #$i: $(tail -2 $OUT/${label}_$i.log | tr '\n' ' ')"
  done
done
