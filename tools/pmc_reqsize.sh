#!/bin/bash
# Read-request sizes at the L2's memory side (TCC_EA0_RDREQ by 32 / 64 / 128 B) and L2 hit / miss counts per
# kernel: calibrates FETCH_SIZE for access widths other than 16-B streaming (MI355X_MICROARCH.md: FETCH_SIZE
# halves wide streaming reads; other widths uncalibrated). One counter group per rocprofv3 run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r1}
OUT=gpurun_out/pmcreq_${TAG}
mkdir -p $OUT
REGEX='k_tile_raster|k_bwd|k_bin|k_vgrad|k_rt_vgrad|k_shade'
CMD="${PMC_CMD:-python bench.py --no-cpu-baseline --no-fragment-pass --no-secondary --steps 3 --warmup 1}"
i=0
for grp in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "$REGEX" -d $OUT/p$i -o run --output-format csv -- $CMD > $OUT/p$i.log 2>&1 || { echo "PMC pass $i failed"; tail -20 $OUT/p$i.log; exit 1; }
done
python tools/pmc_summary.py $OUT > /dev/null
