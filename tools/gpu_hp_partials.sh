#!/bin/bash
# GPU-box side (gpurun -- bash tools/gpu_hp_partials.sh CASE...): per-splat backward sums of each parity case
# (tools/hp_partials.py gpu) into gpurun_out/hp_partials/CASE.pt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/hp_partials
for c in "$@"; do
  timeout -k 10 300 python3 -u tools/hp_partials.py gpu $c gpurun_out/hp_partials/$c.pt || exit 1
done
