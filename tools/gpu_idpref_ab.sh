#!/bin/bash
# GPU-box side: the forward's next-batch id prefetch into LDS (tools/build_variant.sh idpref -DGSTEX_FWD_IDPREF=1):
# raster parity / deep-window / fused tests through the variant, then the cfg3 raster-loop A/B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r06_idpref
GSTEX_LIB=scratch/idpref/libgstex_hip.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_deep.py \
  tests/test_gpu_fused.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_idpref/tests.log 2>&1; rc=$?
echo "tests rc $rc: $(tail -1 gpurun_out/r06_idpref/tests.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/r06_idpref/tests.log; exit 1; }
bash tools/gpu_loop_ab.sh r06_idpref/loop base= idpref=GSTEX_LIB=scratch/idpref/libgstex_hip.so
