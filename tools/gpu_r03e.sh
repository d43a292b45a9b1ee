#!/bin/bash
# GPU-box side: the multi-rank paths with the deferred texel update -- the rehearsal at world 2 (gloo collectives,
# the box's one GPU shared) and bench.py itself under torchrun at world 2 (the driver's N > 1 line, gloo here).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r03; mkdir -p $OUT
GSTEX_DIST_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29612 tools/dist_rehearsal.py --defer-texture > $OUT/dist_rehearsal_w2_defer.log 2>&1
rc=$?; tail -1 $OUT/dist_rehearsal_w2_defer.log
[ $rc -eq 0 ] || { echo "rehearsal rc=$rc"; tail -30 $OUT/dist_rehearsal_w2_defer.log; exit 1; }
GSTEX_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --steps 6 --warmup 3 > $OUT/bench_w2_gloo.log 2>&1
rc=$?; tail -1 $OUT/bench_w2_gloo.log | cut -c1-300
[ $rc -eq 0 ] || { echo "bench w2 rc=$rc"; tail -30 $OUT/bench_w2_gloo.log; exit 1; }
