#!/bin/bash
# A/B of experiment builds: bench (render + fragments) per variant. Usage: gpu_variants.sh TAG base exp/a.so exp/b.so ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; shift
for v in "$@"; do
  if [ "$v" = base ]; then lib=""; else lib="$v"; fi
  n=$(basename "$v" .so)
  MI355R_LIB=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --steps 50 --warmup 10 $BENCH_ARGS > gpurun_out/var_${TAG}_${n}.json 2> gpurun_out/var_${TAG}_${n}.err || { echo "FAILED $n"; tail -20 gpurun_out/var_${TAG}_${n}.err; exit 1; }
  MI355R_LIB=$lib timeout -k 10 120 python bench.py --mode fragments --steps 50 --warmup 10 $BENCH_ARGS > gpurun_out/varf_${TAG}_${n}.json 2> gpurun_out/varf_${TAG}_${n}.err || { echo "FAILED frag $n"; tail -20 gpurun_out/varf_${TAG}_${n}.err; exit 1; }
  python - "$n" gpurun_out/var_${TAG}_${n}.json gpurun_out/varf_${TAG}_${n}.json <<'PY'
import json, sys
r = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1]); f = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
ks = {k: v["avg_us"] for k, v in r["kernels"].items()}
fk = {k: v["avg_us"] for k, v in f["kernels"].items()}
print(f"{sys.argv[1]:>10}: render {r['value']:9.1f} fps {r['ms_per_step']*1e3:6.1f} us | frag {f['value']:9.1f} fps {f['ms_per_step']*1e3:6.1f} us | r {ks} | f {fk}")
PY
done
