#!/bin/bash
# Phase stamps (MR_PROF build in exp/prof.so: python tools/build_variant.py prof -DMR_PROF) of the tile
# raster (render and fragment modes) and the fused backward.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
export MI355R_LIB=$PWD/exp/prof.so
TAG=${1:-s}
timeout -k 10 200 python tools/raster_stamps.py > gpurun_out/rstamp_render_${TAG}.log 2>&1 && \
timeout -k 10 200 python tools/raster_stamps.py frag > gpurun_out/rstamp_frag_${TAG}.log 2>&1 && \
timeout -k 10 200 python tools/bwd_stamps.py > gpurun_out/bstamp_${TAG}.log 2>&1
rc=$?
tail -12 gpurun_out/rstamp_render_${TAG}.log gpurun_out/rstamp_frag_${TAG}.log gpurun_out/bstamp_${TAG}.log
exit $rc
