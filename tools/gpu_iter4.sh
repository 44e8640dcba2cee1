#!/bin/bash
# Iteration: GPU parity suite, headline bench, fragment-pass bench and soft-path bench (no CPU baselines).
# Usage: tools/gpu_iter4.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-it}
bash tools/gpu_iter3.sh "$TAG" || exit $?
timeout -k 10 120 python bench.py --mode fragments --no-cpu-baseline > gpurun_out/benchf_${TAG}.json 2> gpurun_out/benchf_${TAG}.err || { echo "FRAG BENCH FAILED"; tail -20 gpurun_out/benchf_${TAG}.err; exit 1; }
timeout -k 10 200 python bench.py --mode soft --size 128 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/benchs_${TAG}.json 2> gpurun_out/benchs_${TAG}.err || { echo "SOFT BENCH FAILED"; tail -20 gpurun_out/benchs_${TAG}.err; exit 1; }
python - "$TAG" <<'PY'
import json, sys
for m in ("benchf", "benchs"):
    d = json.loads(open(f"gpurun_out/{m}_{sys.argv[1]}.json").read().strip().splitlines()[-1])
    print(m, "value", d["value"], "ms", d["ms_per_step"], {k: v["avg_us"] for k, v in d["kernels"].items()})
PY
