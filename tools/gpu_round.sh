#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprof kernel trace of the bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r1}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1 || { echo "PYTEST FAILED"; tail -40 gpurun_out/pytest_${TAG}.log; exit 1; }
tail -3 gpurun_out/pytest_${TAG}.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 || { echo "SMOKE FAILED"; tail -30 gpurun_out/smoke_${TAG}.log; exit 1; }
cat gpurun_out/smoke_${TAG}.log | tail -2
timeout -k 10 400 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { echo "BENCH FAILED"; tail -30 gpurun_out/bench_${TAG}.err; exit 1; }
cat gpurun_out/bench_${TAG}.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/prof_${TAG}.log 2>&1 || { echo "ROCPROF FAILED"; tail -30 gpurun_out/prof_${TAG}.log; exit 1; }
find gpurun_out/prof_${TAG} -name "*stats*" | head
