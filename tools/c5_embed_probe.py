"""Why the C5 step embedded in the default bench run (secondary_steps, after the headline, the fragment pass and
C3) is slower than bench.py --mode c5 alone: C5 alone twice, then after C3, then after C3 with Python's cyclic
GC frozen; or (--after-headline) alone, after the headline line, after the headline and C3. Experiments only (GPU):
python tools/c5_embed_probe.py [--after-headline]"""
import argparse
import gc
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(0)
    base = dict(gpus=1, steps=20, warmup=8, views=5, size=1024, mesh="cow", no_cpu_baseline=True,
                no_fragment_pass=True, cpu_views=2, no_secondary=True, eager=False, texture="uv", mode="c5")
    c5 = argparse.Namespace(**base)
    pose = argparse.Namespace(**{**base, "size": 512, "views": 64, "steps": 30, "warmup": 10, "mode": "pose"})
    res = {}

    def run(tag):
        torch.cuda.empty_cache()
        e = bench.bench_c5(c5, dev, 1, 0, embed=True)
        res[tag] = {"frames_per_s": e["frames_per_s"], "ms_per_step": e["ms_per_step"],
                    "host_us": e["host_us_per_render_call"], "gc_counts": gc.get_count(),
                    "gc_objects": len(gc.get_objects())}
        print(tag, json.dumps(res[tag]), flush=True)

    if "--after-headline" in sys.argv:  # the default line's order: headline (HIP graph), fragment pass, C3, C5
        run("alone")
        argv = sys.argv
        sys.argv = ["bench.py", "--no-secondary", "--no-cpu-baseline", "--steps", "20", "--warmup", "5"]
        bench.main()
        sys.argv = argv
        gc.collect()
        run("after_headline")
        torch.cuda.empty_cache()
        bench.bench_pose(pose, dev, 1, 0, embed=True)
        gc.collect()
        run("after_headline_pose")
        print(json.dumps(res))
        return
    run("alone_1")
    run("alone_2")
    torch.cuda.empty_cache()
    bench.bench_pose(pose, dev, 1, 0, embed=True)
    run("after_pose")
    gc.collect()
    gc.freeze()
    run("after_pose_gc_frozen")
    gc.unfreeze()
    gc.disable()
    run("after_pose_gc_disabled")
    gc.enable()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
