#!/bin/bash
# Round-4 GPU iteration: parity tests (optional -k filter in $2), the default bench line (with its
# fragment_pass object) and a rocprofv3 kernel trace of the fragment pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r4}
K=${2:-}
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread "${KA[@]}" > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|ERROR" gpurun_out/pytest_${TAG}.log | tail -8
grep -E "^(FAILED|ERROR)" gpurun_out/pytest_${TAG}.log | head -20
# test failures (rc 1) still let the benches run; a timeout / abort / fault ends the call here
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { tail -20 gpurun_out/bench_${TAG}.err; exit 1; }
python - gpurun_out/bench_${TAG}.json <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("render", d["value"], d["ms_per_step"], {k:v["avg_us"] for k,v in d["kernels"].items()})
print("fragment_pass", json.dumps(d.get("fragment_pass")))
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_frag_${TAG} -o run --output-format csv -- python bench.py --mode fragments --steps 20 --warmup 5 > gpurun_out/prof_frag_${TAG}.log 2>&1 || exit 1
python - gpurun_out/prof_frag_${TAG}/run_kernel_stats.csv <<'PY'
import csv,sys
for r in sorted(csv.DictReader(open(sys.argv[1])), key=lambda r:-float(r['TotalDurationNs']))[:6]:
    print(r['Calls'], round(float(r['AverageNs'])/1e3,2), r['Name'][:60])
PY
timeout -k 10 300 python bench.py --mode pose --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/pose_${TAG}.json 2> gpurun_out/pose_${TAG}.err || { tail -20 gpurun_out/pose_${TAG}.err; exit 1; }
python -c "import json,sys; d=json.loads(open('gpurun_out/pose_${TAG}.json').read().strip().splitlines()[-1]); print('pose', d['value'], d['ms_per_step'])"
timeout -k 10 300 python bench.py --mode c5 --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/c5_${TAG}.json 2> gpurun_out/c5_${TAG}.err || { tail -20 gpurun_out/c5_${TAG}.err; exit 1; }
python -c "import json,sys; d=json.loads(open('gpurun_out/c5_${TAG}.json').read().strip().splitlines()[-1]); print('c5', d['value'], d['ms_per_step'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
if [ -f exp/fmax64k.so ]; then
MI355R_LIB=exp/fmax64k.so timeout -k 10 300 python bench.py --mode c5 --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/c5old_${TAG}.json 2> gpurun_out/c5old_${TAG}.err || { tail -20 gpurun_out/c5old_${TAG}.err; exit 1; }
python -c "import json,sys; d=json.loads(open('gpurun_out/c5old_${TAG}.json').read().strip().splitlines()[-1]); print('c5 (count-scan)', d['value'], d['ms_per_step'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
fi
