#!/bin/bash
# GPU-box side: the one-launch backward unit order and the 16-wave tile ranking against the kernels before them.
# scratch/old is the previous source built as a variant: git diff -R --relative=gstex_amd/csrc gstex_amd/csrc >
# scratch/old.patch && PATCH=scratch/old.patch tools/build_variant.sh old (before committing the change).  Runs the
# parity / fused / trainer / deep-window tests on the new build, then rocprofv3 kernel stats over a short bench, new vs old.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r06_unit
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_trainer_sync.py tests/test_gpu_deep.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_unit/tests.log 2>&1; rc=$?
echo "tests rc $rc: $(tail -1 gpurun_out/r06_unit/tests.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/r06_unit/tests.log; exit 1; }
KERNELS='unit_|tile_rank|raster_bwd|raster_fwd' BENCH=1 bash tools/gpu_kernel_ab.sh r06_unit/ab new= old=GSTEX_LIB=scratch/old/libgstex_hip.so
