#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}/tools/micro"
export TMPDIR=/tmp
OUT=../../gpurun_out/pmc_micro
mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_WR SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT" \
           "WRITE_SIZE" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -k 5 120 rocprofv3 --pmc $grp --kernel-include-regex "k_raster|k_strip" -d $OUT/a$i -o run --output-format csv -- ./rc 1 1 64 > $OUT/a$i.log 2>&1 || { echo fail a$i; tail $OUT/a$i.log; exit 1; }
  timeout -k 5 120 rocprofv3 --pmc $grp --kernel-include-regex "k_strip" -d $OUT/b$i -o run --output-format csv -- ./wave_turnover > $OUT/b$i.log 2>&1 || { echo fail b$i; tail $OUT/b$i.log; exit 1; }
done
cd ../..
python tools/pmc_summary.py gpurun_out/pmc_micro > /dev/null
python - <<'PY'
import json
d = json.load(open("gpurun_out/pmc_micro/summary.json"))
for k, v in d.items():
    print(k[:60], {a: round(b) for a, b in v.items()})
PY
