#!/bin/bash
# Round-4 iteration: full GPU tests, default bench line, pose bench under a rocprofv3 kernel trace,
# C5 line, then interleaved A/B of the banding policy (render, fragments).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r4g}
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/pytest_${TAG}.log | tail -3
grep -E "^(FAILED|ERROR)" gpurun_out/pytest_${TAG}.log | head -20
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { tail -20 gpurun_out/bench_${TAG}.err; exit 1; }
python - gpurun_out/bench_${TAG}.json <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("render", d["value"], d["ms_per_step"], {k:v["avg_us"] for k,v in d["kernels"].items()})
fp=d.get("fragment_pass") or {}
print("fragment_pass", fp.get("frames_per_s"), fp.get("pass_us"), fp.get("frac"), fp.get("kernel_us"))
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pose_${TAG} -o run --output-format csv -- python bench.py --mode pose --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/prof_pose_${TAG}.log 2>&1 || { tail -20 gpurun_out/prof_pose_${TAG}.log; exit 1; }
python - gpurun_out/prof_pose_${TAG}/run_kernel_stats.csv <<'PY'
import csv,sys
rows=sorted(csv.DictReader(open(sys.argv[1])), key=lambda r:-float(r['TotalDurationNs']))
print("pose kernels", sum(float(r['TotalDurationNs']) for r in rows)/1e3, "us total")
for r in rows[:14]:
    print(r['Calls'], round(float(r['AverageNs'])/1e3,2), round(float(r['TotalDurationNs'])/1e3,1), r['Name'][:70])
PY
timeout -k 10 300 python bench.py --mode pose --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/pose_${TAG}.json 2> gpurun_out/pose_${TAG}.err || { tail -20 gpurun_out/pose_${TAG}.err; exit 1; }
python -c "import json,sys; d=json.loads(open('gpurun_out/pose_${TAG}.json').read().strip().splitlines()[-1]); print('pose', d['value'], d['ms_per_step'])"
timeout -k 10 300 python bench.py --mode c5 --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/c5_${TAG}.json 2> gpurun_out/c5_${TAG}.err || { tail -20 gpurun_out/c5_${TAG}.err; exit 1; }
python -c "import json,sys; d=json.loads(open('gpurun_out/c5_${TAG}.json').read().strip().splitlines()[-1]); print('c5', d['value'], d['ms_per_step'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
[ -n "$AB_R" ] && { bash tools/gpu_ab_r4.sh ${TAG}r "" $AB_R || exit 1; }
[ -n "$AB_F" ] && { bash tools/gpu_ab_r4.sh ${TAG}f "--mode fragments" $AB_F || exit 1; }
echo done
if [ -n "$CPROF" ]; then
  MR_BENCH_CPROFILE=gpurun_out/pose_cprof_${TAG}.txt timeout -k 10 300 python bench.py --mode pose --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/pose_cp_${TAG}.json 2> gpurun_out/pose_cp_${TAG}.err || { tail -20 gpurun_out/pose_cp_${TAG}.err; exit 1; }
  head -60 gpurun_out/pose_cprof_${TAG}.txt
fi
if [ -n "$CPROF5" ]; then
  MR_BENCH_CPROFILE=gpurun_out/c5_cprof_${TAG}.txt timeout -k 10 300 python bench.py --mode c5 --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/c5_cp_${TAG}.json 2> gpurun_out/c5_cp_${TAG}.err || { tail -20 gpurun_out/c5_cp_${TAG}.err; exit 1; }
  head -70 gpurun_out/c5_cprof_${TAG}.txt
fi
