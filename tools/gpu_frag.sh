set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --mode fragments --steps 50 --warmup 10 > gpurun_out/frag_r2c.json 2> gpurun_out/frag_r2c.err && cat gpurun_out/frag_r2c.json && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_frag_r2c -o run --output-format csv -- python bench.py --mode fragments --steps 20 --warmup 5 > gpurun_out/prof_frag_r2c.log 2>&1 && \
timeout -k 10 300 python bench.py --mesh dolphin --size 1024 --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/c4_r2c.json 2> gpurun_out/c4_r2c.err && cat gpurun_out/c4_r2c.json
