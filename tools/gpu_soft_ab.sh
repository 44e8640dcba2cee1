#!/bin/bash
# A/B of the K-deep soft path (bench.py --mode soft): base library vs experiment builds given as args.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = base ]; then lib=""; else lib="$v"; fi
  MI355R_LIB=$lib timeout -k 10 200 python bench.py --mode soft --size 128 --steps 20 --warmup 5 > gpurun_out/softab.json 2> gpurun_out/softab.err || { tail -5 gpurun_out/softab.err; exit 1; }
  python -c "import json; r=json.loads(open('gpurun_out/softab.json').read().strip().splitlines()[-1]); print('$v', r['value'], r['ms_per_step'], {k: v['avg_us'] for k, v in r['kernels'].items()})"
done
