#!/bin/bash
# GPU-box side: the count kernel's staggered range reservation (tools/build_variant.sh stagger -DGSTEX_COUNT_STAGGER=1):
# the binning parity tests through the variant, then rocprofv3 kernel stats of the binning kernels, default vs variant.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r06_count
GSTEX_LIB=scratch/stagger/libgstex_hip.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k "bin or tile or unit" \
  -x -q --timeout 120 --timeout-method thread > gpurun_out/r06_count/tests.log 2>&1; rc=$?
echo "tests rc $rc: $(tail -1 gpurun_out/r06_count/tests.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/r06_count/tests.log; exit 1; }
KERNELS='count_lds|place|tile_sort|scan_single' bash tools/gpu_kernel_ab.sh r06_count/ab base= stagger=GSTEX_LIB=scratch/stagger/libgstex_hip.so
