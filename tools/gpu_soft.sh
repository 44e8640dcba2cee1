#!/bin/bash
# Soft-rasterization bench line + rocprofv3 kernel stats (tag $1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-s}
timeout -k 10 300 python bench.py --mode soft --size 128 --steps 20 --warmup 5 > gpurun_out/soft_${TAG}.json 2> gpurun_out/soft_${TAG}.err && cat gpurun_out/soft_${TAG}.json && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_soft_${TAG} -o run --output-format csv -- python bench.py --mode soft --size 128 --steps 10 --warmup 3 > gpurun_out/prof_soft_${TAG}.log 2>&1
