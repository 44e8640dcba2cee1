#!/bin/bash
# Round-4 baseline: headline, fragment and pose benches + a rocprofv3 kernel trace of the pose step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r4a}
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err && cat gpurun_out/bench_${TAG}.json | cut -c1-400 && \
timeout -k 10 300 python bench.py --mode fragments --steps 50 --warmup 10 > gpurun_out/frag_${TAG}.json 2> gpurun_out/frag_${TAG}.err && cat gpurun_out/frag_${TAG}.json | cut -c1-600 && \
timeout -k 10 300 python bench.py --mode pose --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/pose_${TAG}.json 2> gpurun_out/pose_${TAG}.err && cat gpurun_out/pose_${TAG}.json | cut -c1-400 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pose_${TAG} -o run --output-format csv -- python bench.py --mode pose --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/prof_pose_${TAG}.log 2>&1 && \
find gpurun_out/prof_pose_${TAG} -name "*stats*"
