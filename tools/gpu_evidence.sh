#!/bin/bash
# Evidence session (tag $1): GPU parity tests, smoke, every bench line (render with its fragment_pass and CPU
# baseline, fragments, soft, pose, C4 gather, C5), rocprofv3 kernel stats of each, the 2-rank rehearsal.
# PMC passes: tools/pmc_profile.sh (separate call).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-ev}
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/pytest_${TAG}.log | tail -2
grep -E "^(FAILED|ERROR)" gpurun_out/pytest_${TAG}.log | head -20
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 || { echo "SMOKE FAILED"; tail -20 gpurun_out/smoke_${TAG}.log; exit 1; }
tail -2 gpurun_out/smoke_${TAG}.log
run() {  # name, timeout, args...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to python bench.py "$@" > gpurun_out/${name}_${TAG}.json 2> gpurun_out/${name}_${TAG}.err || { echo "$name FAILED"; tail -20 gpurun_out/${name}_${TAG}.err; return 1; }
  python - gpurun_out/${name}_${TAG}.json $name <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
fp=d.get("fragment_pass") or {}
print(sys.argv[2], d["value"], d["unit"], d["ms_per_step"], "cpu", (d.get("cpu_baseline") or {}).get("value"), "roof", (d.get("roofline") or {}).get("frac"), "frag", fp.get("frames_per_s"), fp.get("frac"), fp.get("kernel_sum_frac"))
PY
}
prof() {  # name, args...
  local name=$1; shift
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${name}_${TAG} -o run --output-format csv -- python bench.py --no-cpu-baseline "$@" > gpurun_out/prof_${name}_${TAG}.log 2>&1 || { echo "ROCPROF $name FAILED"; tail -20 gpurun_out/prof_${name}_${TAG}.log; return 1; }
  python - gpurun_out/prof_${name}_${TAG}/run_kernel_stats.csv $name <<'PY'
import csv,sys
rows=sorted(csv.DictReader(open(sys.argv[1])), key=lambda r:-float(r['TotalDurationNs']))
print(sys.argv[2], 'kernels:', ', '.join('%s %.1f' % (r['Name'].replace('void ','').split('(')[0][:28], float(r['AverageNs'])/1e3) for r in rows[:8]))
PY
}
run bench 400 && prof render --no-fragment-pass --no-secondary --steps 20 --warmup 5 && \
run frag 300 --mode fragments --steps 50 --warmup 10 && prof frag --mode fragments --steps 20 --warmup 5 && \
run soft 400 --mode soft --size 128 && prof soft --mode soft --size 128 --steps 10 --warmup 3 && \
run pose 400 --mode pose --steps 20 --warmup 5 && prof pose --mode pose --steps 20 --warmup 5 && \
run c5 400 --mode c5 --steps 60 --warmup 10 && prof c5 --mode c5 --steps 10 --warmup 3 && \
run c4 300 --mode gather --mesh dolphin --size 1024 --views 64 --no-cpu-baseline --steps 20 --warmup 5 && \
MR_BENCH_REHEARSE=1 run rehearse 300 --gpus 2 --no-cpu-baseline --no-fragment-pass --steps 10 --warmup 3 && \
python -c "import json; d=json.loads(open('gpurun_out/rehearse_${TAG}.json').read().strip().splitlines()[-1]); print('rehearse', d.get('n_gpus'), d.get('allreduce_us'), d.get('allreduce_overlapped_with_forward'), d.get('allreduce_check'))"
echo done
