#!/bin/bash
# Round-5 split-backward experiment on the GPU box: parity of the split path, then the raster loop (cfg3, photometric)
# with the default and the split backward interleaved, then a kernel trace of each (rocprofv3), then (optional) the
# slow tests.  Outputs under gpurun_out/split/.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/split; mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_split.py tests/test_gpu_callseq.py -v -s --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
grep -E "passed|failed" $OUT/tests.log | tail -1
for i in 1 2; do
  timeout -k 10 120 python3 tools/raster_loop.py --photometric --no-geometry --iters 20 > $OUT/loop_default_$i.log 2>&1 || exit 1
  echo "default: $(tail -1 $OUT/loop_default_$i.log)"
  GSTEX_BWD_SPLIT=1 timeout -k 10 120 python3 tools/raster_loop.py --photometric --no-geometry --iters 20 > $OUT/loop_split_$i.log 2>&1 || exit 1
  echo "split:   $(tail -1 $OUT/loop_split_$i.log)"
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_default -o run -- python3 tools/raster_loop.py --photometric --no-geometry --iters 10 > $OUT/trace_default.log 2>&1 || exit 1
GSTEX_BWD_SPLIT=1 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_split -o run -- python3 tools/raster_loop.py --photometric --no-geometry --iters 10 > $OUT/trace_split.log 2>&1 || exit 1
if [ -n "$PMC" ]; then
  GSTEX_BWD_SPLIT=1 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/pmc_split -o run -- python3 tools/raster_loop.py --photometric --no-geometry --iters 3 > $OUT/pmc_split.log 2>&1 || exit 1
  GSTEX_BWD_SPLIT=1 timeout -s KILL 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr --output-format csv -d $OUT/pmc_split_tcp -o run -- python3 tools/raster_loop.py --photometric --no-geometry --iters 3 > $OUT/pmc_split_tcp.log 2>&1 || echo "tcp pass failed"
  timeout -s KILL 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr --output-format csv -d $OUT/pmc_default_tcp -o run -- python3 tools/raster_loop.py --photometric --no-geometry --iters 3 > $OUT/pmc_default_tcp.log 2>&1 || echo "tcp pass failed"
fi
if [ -n "$HOSTPROF" ]; then
  timeout -k 10 300 python3 -u tools/host_profile.py > $OUT/host_profile.log 2>&1 || { tail -20 $OUT/host_profile.log; exit 1; }
  head -60 $OUT/host_profile.log
fi
if [ -n "$SLOW" ]; then
  timeout -k 10 900 python3 -u -m pytest tests/test_gpu_trajectory.py -v -s --timeout 900 --timeout-method thread > $OUT/trajectory.log 2>&1; tail -25 $OUT/trajectory.log
fi
echo done
