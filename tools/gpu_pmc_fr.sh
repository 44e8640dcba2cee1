#!/bin/bash
# k_face_reduce wave life vs kernel length: one PMC pass per counter group (no tracing domains).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-fr}
OUT=gpurun_out/pmc_${TAG}
mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" "FETCH_SIZE" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex 'k_face_reduce|k_bwd_fused|k_bin_view' -d $OUT/p$i -o run --output-format csv -- python bench.py --no-cpu-baseline --no-fragment-pass --steps 3 --warmup 1 > $OUT/p$i.log 2>&1 || { echo "PMC pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python tools/pmc_summary.py $OUT
