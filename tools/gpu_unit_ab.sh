cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r06_unit
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_trainer_sync.py tests/test_gpu_deep.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_unit/tests.log 2>&1; rc=$?
echo "tests rc $rc: $(tail -1 gpurun_out/r06_unit/tests.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/r06_unit/tests.log; exit 1; }
KERNELS='unit_|tile_rank|raster_bwd|raster_fwd' BENCH=1 bash tools/gpu_kernel_ab.sh r06_unit/ab new= old=GSTEX_LIB=scratch/old/libgstex_hip.so
