#!/bin/bash
# GPU-box side (gpurun -- bash tools/gpu_hp_pairs.sh CASE [GID...]): per-pair backward records of the parity case
# (tools/hp_pairs.py gpu, the scratch/pairs build) into gpurun_out/hp_pairs/CASE.pt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/hp_pairs
c=$1; shift
GSTEX_LIB=scratch/pairs/libgstex_hip.so timeout -k 10 300 python3 -u tools/hp_pairs.py gpu $c gpurun_out/hp_pairs/$c.pt "$@" || exit 1
