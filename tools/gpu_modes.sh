set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
export MI355R_LIB=$PWD/exp/prof.so
timeout -k 10 200 python tools/raster_stamps.py > gpurun_out/rstamp_render.log 2>&1
timeout -k 10 200 python tools/raster_stamps.py frag > gpurun_out/rstamp_frag.log 2>&1
timeout -k 10 200 python tools/bwd_stamps.py > gpurun_out/bstamp.log 2>&1
unset MI355R_LIB
timeout -k 10 300 python bench.py --mode gather --mesh dolphin --size 1024 --views 64 --steps 10 --warmup 3 > gpurun_out/b_gather1.json 2> gpurun_out/b_gather1.err
MR_BENCH_REHEARSE=1 timeout -k 10 300 python bench.py --gpus 2 --mode gather --mesh dolphin --size 1024 --views 64 --steps 5 --warmup 2 > gpurun_out/b_gather2.json 2> gpurun_out/b_gather2.err
timeout -k 10 400 python bench.py --mode pose --views 64 --steps 10 --warmup 3 > gpurun_out/b_pose.json 2> gpurun_out/b_pose.err
timeout -k 10 400 python bench.py --mode soft --size 128 --steps 10 --warmup 3 > gpurun_out/b_soft.json 2> gpurun_out/b_soft.err
MR_BENCH_REHEARSE=1 timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b_rehearse2.json 2> gpurun_out/b_rehearse2.err
echo done
