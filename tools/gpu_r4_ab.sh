#!/bin/bash
# Round-4 experiment call: interleaved A/B of exp/ variants on the render, fragment and soft benches,
# then the 2-rank rehearsal of the N > 1 path on the one GPU (gloo) and a rocprofv3 trace of the pose step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-ab}
RV=${RENDER_VARIANTS:-"bwd3 bgwg2 bgwg2b aos"}
FV=${FRAG_VARIANTS:-"bgwg2 bgwg2b aos"}
SV=${SOFT_VARIANTS:-"aos"}
bash tools/gpu_ab_r4.sh ${TAG}r "" $RV || exit 1
bash tools/gpu_ab_r4.sh ${TAG}f "--mode fragments" $FV || exit 1
bash tools/gpu_ab_r4.sh ${TAG}s "--mode soft --size 128" $SV || exit 1
MR_BENCH_REHEARSE=1 timeout -k 10 300 python bench.py --gpus 2 --no-cpu-baseline --no-fragment-pass --steps 10 --warmup 3 > gpurun_out/rehearse_${TAG}.json 2> gpurun_out/rehearse_${TAG}.err || { tail -20 gpurun_out/rehearse_${TAG}.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/rehearse_${TAG}.json').read().strip().splitlines()[-1]); print('rehearse', d['n_gpus'], d['value'], d['allreduce_us'], d['allreduce_check'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pose_${TAG} -o run --output-format csv -- python bench.py --mode pose --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/prof_pose_${TAG}.log 2>&1 || exit 1
echo done
