#!/bin/bash
# GPU-box side: the forward's next-batch record cache warming (PATCH=tools/variants/fwd_recwarm.patch
# tools/build_variant.sh recwarm -DGSTEX_FWD_RECWARM=1):
# raster parity / deep-window / fused tests through the variant, then the cfg3 raster-loop A/B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r06_recwarm
GSTEX_LIB=scratch/recwarm/libgstex_hip.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_deep.py \
  tests/test_gpu_fused.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_recwarm/tests.log 2>&1; rc=$?
echo "tests rc $rc: $(tail -1 gpurun_out/r06_recwarm/tests.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/r06_recwarm/tests.log; exit 1; }
bash tools/gpu_loop_ab.sh r06_recwarm/loop base= recwarm=GSTEX_LIB=scratch/recwarm/libgstex_hip.so
