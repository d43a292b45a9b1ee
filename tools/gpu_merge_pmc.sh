#!/bin/bash
# GPU-box side: SQ counter passes (tools/gpu_pmc.sh) for the default build and the merged-backward variants, then the
# raster-loop timing of the record-only variant (mskip: forward contributing-lane record + empty-visit skip); the
# variants are built from tools/variants/bwd_merge.patch (tools/build_variant.sh with PATCH=...).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=merge_base bash tools/gpu_pmc.sh > /dev/null 2>&1 && \
TAG=merge_m6 LIB=scratch/merge6/libgstex_hip.so bash tools/gpu_pmc.sh > /dev/null 2>&1 && \
TAG=merge_skip LIB=scratch/mskip/libgstex_hip.so bash tools/gpu_pmc.sh > /dev/null 2>&1 && \
bash tools/gpu_loop_ab.sh r06_merge3/loop base= mskip=GSTEX_LIB=scratch/mskip/libgstex_hip.so
