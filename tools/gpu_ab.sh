#!/bin/bash
# GPU iteration: parity tests, then render + fragment + C4 bench lines (no CPU baseline).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-ab}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1 || { echo "PYTEST FAILED"; grep -E "FAILED|Error|error|assert" gpurun_out/pytest_${TAG}.log | head -30; tail -30 gpurun_out/pytest_${TAG}.log; exit 1; }
tail -2 gpurun_out/pytest_${TAG}.log
bash tools/gpu_variants.sh $TAG base || exit 1
timeout -k 10 200 python bench.py --mesh dolphin --size 1024 --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/c4_${TAG}.json 2> gpurun_out/c4_${TAG}.err || { echo "C4 FAILED"; tail -20 gpurun_out/c4_${TAG}.err; exit 1; }
python -c "import json,sys; r=json.loads(open('gpurun_out/c4_${TAG}.json').read().strip().splitlines()[-1]); print('C4', r['value'], r['ms_per_step'], {k: v['avg_us'] for k, v in r['kernels'].items()})"
