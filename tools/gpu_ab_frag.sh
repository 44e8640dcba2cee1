#!/bin/bash
# Fragment-pass A/B of library builds: tools/gpu_ab_frag.sh TAG base exp/a.so ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; shift
for rep in 1 2; do
for v in "$@"; do
  if [ "$v" = base ]; then lib=""; else lib="$v"; fi
  n=$(basename "$v" .so)
  MI355R_LIB=$lib timeout -k 10 120 python bench.py --mode fragments --no-cpu-baseline --steps 50 --warmup 10 > gpurun_out/abf_${TAG}_${n}.json 2> gpurun_out/abf_${TAG}_${n}.err || { echo "FAILED $n"; tail -20 gpurun_out/abf_${TAG}_${n}.err; exit 1; }
  python - "$n" gpurun_out/abf_${TAG}_${n}.json <<'PY'
import json, sys
r = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ks = {k: v["avg_us"] for k, v in r["kernels"].items()}
print(f"{sys.argv[1]:>10}: {r['value']:9.1f} fps {r['ms_per_step']*1e3:6.1f} us | {ks}")
PY
done
done
