#!/bin/bash
# Stall/latency counter passes over the raster-only loop (one rocprofv3 --pmc run per pass, <= 8 SQ counters).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc; mkdir -p $OUT
LIB=${LIB:-gstex_amd/libgstex_hip.so}
i=0
for pass in "SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY" \
            "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_WAIT_INST_ANY SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU"; do
  i=$((i+1))
  GSTEX_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d $OUT/p$i -o run -- python3 tools/raster_loop.py --photometric --iters 3 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo done
