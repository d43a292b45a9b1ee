#!/bin/bash
# cfg4's 8-rank sharding rehearsed on one GPU: GStexTrainer + GradSync + HIP kernels at world 8 (gloo carries the
# collectives), deferred texel update (the bench default: head first, tail in pieces) and the plain exchange.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/s10; mkdir -p $OUT
GSTEX_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29614 tools/dist_rehearsal.py --defer-texture > $OUT/dist_rehearsal_w8_defer.log 2>&1
rc=$?; tail -1 $OUT/dist_rehearsal_w8_defer.log
[ $rc -eq 0 ] || { echo "rehearsal w8 defer rc=$rc"; grep -v "socket.cpp\|Gloo" $OUT/dist_rehearsal_w8_defer.log | tail -30; exit 1; }
GSTEX_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29615 tools/dist_rehearsal.py > $OUT/dist_rehearsal_w8.log 2>&1
rc=$?; tail -1 $OUT/dist_rehearsal_w8.log
[ $rc -eq 0 ] || { echo "rehearsal w8 rc=$rc"; grep -v "socket.cpp\|Gloo" $OUT/dist_rehearsal_w8.log | tail -30; exit 1; }
