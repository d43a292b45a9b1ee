#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration passes (tools/fetch_calibrate.hip, built into scratch/fetchcal on the CPU side).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/fetchcal; mkdir -p $OUT
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- ./scratch/fetchcal > $OUT/trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- ./scratch/fetchcal > $OUT/fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- ./scratch/fetchcal > $OUT/write.log 2>&1 || exit 1
echo fetchcal done
