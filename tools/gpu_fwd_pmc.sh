#!/bin/bash
# Forward stall breakdown at cfg3 (raster loop, photometric variant): where the raster forward's waves spend their
# cycles (issue vs waits, LDS, scalar unit), one rocprofv3 --pmc pass per counter group (per-pass block limits).
# Usage (GPU box): bash tools/gpu_fwd_pmc.sh [tag]; results under gpurun_out/fwdpmc_<tag>/.
set -o pipefail
TAG=${1:-base}
OUT=gpurun_out/fwdpmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 60 rocprofv3 --list-avail > $OUT/list_avail.txt 2>&1 || echo "list-avail failed"
LOOP="python3 tools/raster_loop.py --photometric --no-geometry --iters 3"
i=0
for grp in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA" \
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM" \
  "SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_EXP SQ_INSTS_SENDMSG"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- $LOOP > $OUT/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "pmc pass $i failed rc=$rc (see $OUT/p$i.log)"
    # a killed / aborted / faulting pass ends the script (an unknown counter is an ordinary error exit)
    case $rc in 124|134|137|139) exit $rc ;; esac
  fi
done
echo "fwd pmc $TAG done"
