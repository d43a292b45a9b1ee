#!/bin/bash
# GPU-box side of an A/B run: raster-only cfg3 loop (photometric upstream grads) for every
# scratch/<variant>/libgstex_hip.so given on the command line (the bench's variant: no geometry outputs), then (optional) stall-counter passes.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/ablate; mkdir -p $OUT
for v in "$@"; do
  GSTEX_LIB=scratch/$v/libgstex_hip.so timeout -k 10 120 python3 tools/raster_loop.py --photometric --no-geometry --iters 20 > $OUT/$v.log 2>&1 || { echo "FAIL $v"; exit 1; }
  echo "$v: $(tail -2 $OUT/$v.log | tr '\n' ' ')"
done
if [ -n "$PMC" ]; then
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv -d $OUT/pmc1 -o run -- python3 tools/raster_loop.py --photometric --iters 3 > $OUT/pmc1.log 2>&1 || { echo "pmc1 failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES --output-format csv -d $OUT/pmc2 -o run -- python3 tools/raster_loop.py --photometric --iters 3 > $OUT/pmc2.log 2>&1 || { echo "pmc2 failed"; exit 1; }
fi
echo done
