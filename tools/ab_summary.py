"""Summarise an interleaved A/B (tools/gpu_ab.sh outputs) into one text table.
python tools/ab_summary.py TAG > profiles/<TAG>_ab.txt"""
import glob
import json
import os
import sys

tag = sys.argv[1]
for path in sorted(glob.glob(f"gpurun_out/ab_{tag}_*_[12].json"), key=lambda p: (p[-6], p)):
    d = json.loads(open(path).read().strip().splitlines()[-1])
    name = os.path.basename(path)[len(f"ab_{tag}_"):-5]
    ks = {k: v["avg_us"] for k, v in d.get("kernels", {}).items()}
    print(f"{name:14s} {d['value']:>10} {d['ms_per_step']:.4f} ms  {ks}")
