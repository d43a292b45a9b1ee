#!/bin/bash
# GPU-box side: the disjoint-visit merged backward experiment (GSTEX_BWD_MERGE; variants merge / merge6 / mstats built
# by PATCH=tools/variants/bwd_merge.patch tools/build_variant.sh, stats by tools/build_variant.sh).  Parity of the merge build (raster parity, deep windows, fused training step), its work counters
# beside the default's, then the cfg3 raster-loop A/B.  Output under gpurun_out/<TAG>/.
TAG=${1:?usage: gpu_merge_ab.sh TAG}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
GSTEX_LIB=scratch/merge/libgstex_hip.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_deep.py tests/test_gpu_fused.py -x -q --timeout 300 --timeout-method thread > $OUT/parity_merge.log 2>&1
rc=$?; echo "merge parity: rc $rc $(grep -E 'passed|failed' $OUT/parity_merge.log | tail -1)"
[ $rc -eq 0 ] || { tail -30 $OUT/parity_merge.log; exit 1; }
for v in stats mstats; do
  GSTEX_LIB=scratch/$v/libgstex_hip.so timeout -k 10 180 python3 -u tools/raster_loop.py --photometric --iters 5 \
    > $OUT/stats_$v.log 2>&1 || { echo "stats $v FAILED"; tail -5 $OUT/stats_$v.log; exit 1; }
  echo "$v: $(grep 'stats/launch' $OUT/stats_$v.log)"
done
bash tools/gpu_loop_ab.sh $TAG/loop base= merge=GSTEX_LIB=scratch/merge/libgstex_hip.so \
  merge6=GSTEX_LIB=scratch/merge6/libgstex_hip.so
