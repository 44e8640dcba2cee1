set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c5prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c5prof/c5 -o run --output-format csv -- python bench.py --mode c5 --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/c5prof/c5.json 2> gpurun_out/c5prof/c5.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c5prof/pose -o run --output-format csv -- python bench.py --mode pose --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/c5prof/pose.json 2> gpurun_out/c5prof/pose.err
