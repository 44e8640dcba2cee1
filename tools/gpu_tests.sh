#!/bin/bash
# GPU parity tests only (optionally a -k filter): python -u, per-test timeout, log under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-t}
shift
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread "$@" > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|\[parity\]|\[determinism\]|passed|failed" gpurun_out/pytest_${TAG}.log | tail -80
exit $rc
