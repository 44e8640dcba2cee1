#!/bin/bash
# Iteration: GPU parity suite (all tests, no -x), then the headline bench (no CPU baseline) with per-kernel
# timings. Usage: tools/gpu_iter3.sh TAG [extra bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-it}
shift
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_${TAG}.log | tail -30
if [ $rc -ne 0 ] && ! grep -qE "[0-9]+ passed" gpurun_out/pytest_${TAG}.log; then echo "pytest aborted rc=$rc"; exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { echo "BENCH FAILED"; tail -20 gpurun_out/bench_${TAG}.err; exit 1; }
python - "$TAG" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/bench_{sys.argv[1]}.json").read().strip().splitlines()[-1])
print("value", d["value"], "ms", d["ms_per_step"], {k: v["avg_us"] for k, v in d["kernels"].items()})
PY
exit $rc
