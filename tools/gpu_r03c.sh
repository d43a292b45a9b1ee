#!/bin/bash
# Rehearsal (first), A/B raster timing of the working tree vs variants and the HEAD tree, then the GPU tests.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r03; mkdir -p $OUT
for W in ${WORLDS:-2 4}; do
  GSTEX_DIST_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $W \
    --master-addr 127.0.0.1 --master-port $((29500 + W)) tools/dist_rehearsal.py > $OUT/dist_rehearsal_w$W.log 2>&1
  rc=$?; tail -1 $OUT/dist_rehearsal_w$W.log
  [ $rc -eq 0 ] || { echo "rehearsal world $W rc=$rc"; tail -30 $OUT/dist_rehearsal_w$W.log; exit 1; }
done
bash tools/gpu_check.sh "$@"
