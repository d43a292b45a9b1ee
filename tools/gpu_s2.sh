#!/bin/bash
# Pair-backward experiment: quadrant-pair census, parity of the pair kernel (GSTEX_LIB variant), raster-loop timings.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/s2; mkdir -p $OUT
timeout -k 10 120 python3 -u tools/pair_union.py > $OUT/pair_union.log 2>&1 || { echo "pair_union FAILED"; tail -20 $OUT/pair_union.log; exit 1; }
cat $OUT/pair_union.log
GSTEX_LIB=scratch/pair512/libgstex_hip.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_deep.py -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/pair_tests.log 2>&1
rc=$?
tail -3 $OUT/pair_tests.log
[ $rc = 0 ] || exit $rc
FILTER="raster_bwd|raster_fwd" timeout -k 10 600 bash tools/gpu_trace_variants.sh head pair pair512 pairv512
