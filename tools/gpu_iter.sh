#!/bin/bash
# GPU iteration: parity tests, per-kernel timings, bench (no CPU baseline). Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-it}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1 || { echo "PYTEST FAILED"; tail -60 gpurun_out/pytest_${TAG}.log; exit 1; }
tail -3 gpurun_out/pytest_${TAG}.log
timeout -k 10 200 python tools/kbench.py --iters 20 > gpurun_out/kbench_${TAG}.log 2>&1 || { echo "KBENCH FAILED"; tail -30 gpurun_out/kbench_${TAG}.log; exit 1; }
tail -2 gpurun_out/kbench_${TAG}.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { echo "BENCH FAILED"; tail -30 gpurun_out/bench_${TAG}.err; exit 1; }
cat gpurun_out/bench_${TAG}.json
