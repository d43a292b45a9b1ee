#!/bin/bash
# The geometry-regularised training mode (cfg5): its GPU test, then the 4-rank rehearsal with it (gloo, one GPU).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/s11; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_geometry.py tests/test_conventions.py -m gpu -x -v --timeout 150 --timeout-method thread > $OUT/geo_tests.log 2>&1
rc=$?; grep -E "passed|failed" $OUT/geo_tests.log | tail -1
[ $rc -eq 0 ] || { grep -E "Error|assert|^E " $OUT/geo_tests.log | head -30; exit 1; }
GSTEX_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29616 tools/dist_rehearsal.py --geo --defer-texture > $OUT/dist_rehearsal_w4_geo.log 2>&1
rc=$?; grep texture_dc $OUT/dist_rehearsal_w4_geo.log; tail -1 $OUT/dist_rehearsal_w4_geo.log
[ $rc -eq 0 ] || { echo "rehearsal rc=$rc"; grep -v "socket.cpp\|Gloo" $OUT/dist_rehearsal_w4_geo.log | tail -30; exit 1; }
GSTEX_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29620 tools/dist_rehearsal.py --geo > $OUT/dist_rehearsal_w4_geo_plain.log 2>&1
rc=$?; grep texture_dc $OUT/dist_rehearsal_w4_geo_plain.log; tail -1 $OUT/dist_rehearsal_w4_geo_plain.log
[ $rc -eq 0 ] || { echo "rehearsal plain rc=$rc"; exit 1; }
