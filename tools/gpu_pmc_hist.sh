#!/bin/bash
# LDS bank conflicts of k_bin_view on the fragment pass for the histogram-copy variants (one PMC pass each,
# kernel trace off), then an interleaved timing A/B of the same variants.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-hc}
shift
for v in base "$@"; do
  if [ "$v" = base ]; then LIB=""; else LIB="exp/$v.so"; fi
  OUT=gpurun_out/pmc_${TAG}_${v}
  mkdir -p $OUT
  MI355R_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS \
    --kernel-include-regex 'k_bin_view|k_bin_rect|k_tile_raster' -d $OUT/p1 -o run --output-format csv -- \
    python bench.py --mode fragments --no-cpu-baseline --steps 3 --warmup 1 > $OUT/p1.log 2>&1 || { echo "PMC $v failed"; tail -5 $OUT/p1.log; exit 1; }
  python tools/pmc_summary.py $OUT > /dev/null && python - $OUT/summary.json $v <<'PY'
import json,sys
d=json.load(open(sys.argv[1]))
for k,v in d.items():
    if 'bin_view' in k or 'bin_rect' in k:
        print(sys.argv[2], k, 'conflict/active = %.3f' % (v['SQ_LDS_BANK_CONFLICT']/max(v['SQ_LDS_IDX_ACTIVE'],1)), {c: round(x) for c,x in v.items()})
PY
done
bash tools/gpu_ab_r4.sh ${TAG}f "--mode fragments" "$@" || exit 1
bash tools/gpu_ab_r4.sh ${TAG}r "" "$@" || exit 1
echo done
