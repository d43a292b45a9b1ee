#!/bin/bash
# Multi-rank paths after the chunked head-first tail: RCCL world-1 trainer tests, the world-2 rehearsal with the
# deferred texel update (gloo, one GPU shared), bench.py under torchrun at world 2 (gloo).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/s8; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_trainer_sync.py -m gpu -x -v --timeout 150 --timeout-method thread > $OUT/trainer_sync.log 2>&1
rc=$?; grep -E "passed|failed" $OUT/trainer_sync.log | tail -1
[ $rc -eq 0 ] || { tail -30 $OUT/trainer_sync.log; exit 1; }
GSTEX_DIST_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29612 tools/dist_rehearsal.py --defer-texture > $OUT/dist_rehearsal_w2_defer.log 2>&1
rc=$?; tail -1 $OUT/dist_rehearsal_w2_defer.log
[ $rc -eq 0 ] || { echo "rehearsal rc=$rc"; tail -30 $OUT/dist_rehearsal_w2_defer.log; exit 1; }
GSTEX_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --steps 6 --warmup 3 > $OUT/bench_w2_gloo.log 2>&1
rc=$?; tail -1 $OUT/bench_w2_gloo.log | cut -c1-300
[ $rc -eq 0 ] || { echo "bench w2 rc=$rc"; tail -30 $OUT/bench_w2_gloo.log; exit 1; }
