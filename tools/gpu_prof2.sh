#!/bin/bash
# rocprofv3 kernel stats of the render step and of the fragment pass (no CPU baseline), tag $1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-p}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/prof_${TAG}.log 2>&1 || { echo "ROCPROF FAILED"; tail -20 gpurun_out/prof_${TAG}.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_frag_${TAG} -o run --output-format csv -- python bench.py --mode fragments --steps 20 --warmup 5 > gpurun_out/prof_frag_${TAG}.log 2>&1 || { echo "ROCPROF FRAG FAILED"; tail -20 gpurun_out/prof_frag_${TAG}.log; exit 1; }
python - "$TAG" <<'PY'
import csv, sys
t = sys.argv[1]
for f in (f"gpurun_out/prof_{t}/run_kernel_stats.csv", f"gpurun_out/prof_frag_{t}/run_kernel_stats.csv"):
    print(f)
    for r in csv.DictReader(open(f)):
        if int(r["Calls"]) >= 10:
            print(f"  {r['Calls']:>5} {float(r['AverageNs'])/1e3:8.2f}  {r['Name'][:90]}")
PY
