#!/bin/bash
# A/B of experiment builds (exp/<name>.so) on the render bench, interleaved: base, v1, v2, ..., repeated twice.
# usage: tools/gpu_ab.sh TAG MODEARGS variant...   (MODEARGS e.g. "--mode fragments")
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; MODEARGS=$2; shift 2
for rep in 1 2; do
  for v in base "$@"; do
    if [ "$v" = base ]; then LIB=""; else LIB="exp/$v.so"; fi
    MI355R_LIB=$LIB timeout -k 10 200 python bench.py $MODEARGS --no-cpu-baseline --no-fragment-pass --no-secondary --steps 50 --warmup 10 > gpurun_out/ab_${TAG}_${v}_${rep}.json 2> gpurun_out/ab_${TAG}_${v}_${rep}.err || { tail -5 gpurun_out/ab_${TAG}_${v}_${rep}.err; exit 1; }
    python - gpurun_out/ab_${TAG}_${v}_${rep}.json "$v" <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["value"], d["ms_per_step"], {k:v["avg_us"] for k,v in d.get("kernels",{}).items()})
PY
  done
done
