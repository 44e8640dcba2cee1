#!/bin/bash
# failing-test recheck + interleaved A/B of the round-4 knobs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r4f}
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "metric_config or c4_dolphin or lazy_zbuf or soft_silhouette_bench or determinism or share_one_raster" > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_${TAG}.log | tail -14
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
bash tools/gpu_ab_r4.sh ${TAG}r "" bwd3 bgwg2 bgwg2b aos bands1 || exit 1
bash tools/gpu_ab_r4.sh ${TAG}f "--mode fragments" bgwg2 bgwg2b aos bands1 || exit 1
bash tools/gpu_ab_r4.sh ${TAG}s "--mode soft --size 128" aos || exit 1
echo done
