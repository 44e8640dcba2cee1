#!/bin/bash
# PMC passes (one counter group per rocprofv3 run; no tracing domains combined with --pmc).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r1}
OUT=gpurun_out/pmc_${TAG}
mkdir -p $OUT
REGEX='k_tile_raster|k_face|k_bwd|k_bin|k_vgrad|k_rt_vgrad|k_vertex|k_shade|k_project|k_rt_reduce|k_fill|k_raster'
CMD="${PMC_CMD:-python bench.py --no-cpu-baseline --no-fragment-pass --no-secondary --steps 3 --warmup 1}"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "$REGEX" -d $OUT/p$i -o run --output-format csv -- $CMD > $OUT/p$i.log 2>&1 || { echo "PMC pass $i failed"; tail -20 $OUT/p$i.log; exit 1; }
done
python tools/pmc_summary.py $OUT
