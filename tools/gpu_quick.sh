#!/bin/bash
# GPU iteration loop: parity tests, per-kernel timings, micro benchmark.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/kbench.py --iters 20 && \
for a in "1 1 64" "4096 1 64" "4096 0 1"; do timeout -k 10 60 tools/micro/rc $a || exit 1; done
