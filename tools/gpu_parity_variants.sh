#!/bin/bash
# GPU-box side: the raster parity / deep-window tests (printed per-gradient errors vs the fp64 oracle) for the default
# build and for every scratch/<variant>/libgstex_hip.so named (tools/build_variant.sh), one log each.
TAG=${1:?usage: gpu_parity_variants.sh TAG [variant ...]}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
for v in default "$@"; do
  if [ "$v" = default ]; then unset GSTEX_LIB; else export GSTEX_LIB=scratch/$v/libgstex_hip.so; fi
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_deep.py tests/test_gpu_parity.py -k "raster or cfg" -v -s \
    --timeout 300 --timeout-method thread > $OUT/parity_$v.log 2>&1
  echo "$v: rc $? $(grep -E 'passed|failed' $OUT/parity_$v.log | tail -1)"
done
