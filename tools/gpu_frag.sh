#!/bin/bash
# Fragment-pass bench + rocprofv3 kernel stats, and the C4 workload bench (tag $1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-f}
timeout -k 10 300 python bench.py --mode fragments --steps 50 --warmup 10 > gpurun_out/frag_${TAG}.json 2> gpurun_out/frag_${TAG}.err && cat gpurun_out/frag_${TAG}.json && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_frag_${TAG} -o run --output-format csv -- python bench.py --mode fragments --steps 20 --warmup 5 > gpurun_out/prof_frag_${TAG}.log 2>&1 && \
timeout -k 10 300 python bench.py --mesh dolphin --size 1024 --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/c4_${TAG}.json 2> gpurun_out/c4_${TAG}.err && cat gpurun_out/c4_${TAG}.json
