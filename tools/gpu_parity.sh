#!/bin/bash
# All GPU parity tests WITHOUT stopping at the first failure (-x off): the full [parity] landscape.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-p}
shift
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread "$@" > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_${TAG}.log | tail -40
exit $rc
