"""Copy one GPU session's evidence from gpurun_out/ into profiles/ (tracked):
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats of `bench.py --steps 20 --warmup 5`
  profiles/<tag>_pmc.json           per-kernel PMC means per dispatch (tools/pmc_profile.sh)
  profiles/<tag>_bench.json         the bench.py JSON line of the same session
  profiles/pmc_traffic.json         HBM bytes per launch (gfx950-corrected) that bench.py reports as
                                    roofline.traffic when its config matches
usage: python tools/collect_profiles.py <tag> [--config cow-512x512-64]"""
import argparse
import json
import os
import re
import shutil

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def short(name):
    n = name.replace("void ", "").split("(")[0].strip()
    m = re.match(r"(k_bwd_fused|k_face_reduce|k_rt_vgrad_a|k_bwd_geom|k_vgrad_a|k_vgrad_b|k_tile_raster|k_bin_count_world|k_bin_fill_world|k_bin_view|k_bin_rect_world|k_bin_rect_fv)<.*>", n)
    if m:
        return {"k_bin_count_world": "k_bin_count", "k_bin_fill_world": "k_bin_fill", "k_bin_rect_world": "k_bin_rect", "k_bin_rect_fv": "k_bin_rect"}.get(m.group(1), m.group(1))
    m = re.match(r"k_shade<(\d+), *\d+>", n)
    return f"k_shade<{m.group(1)}>" if m else re.sub(r"<(true|false)>", "", n)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--config", default="cow-512x512-64")
    a = ap.parse_args()
    out = os.path.join(ROOT, "gpurun_out")
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    shutil.copy(os.path.join(out, f"prof_{a.tag}", "run_kernel_stats.csv"),
                os.path.join(prof, f"{a.tag}_kernel_stats.csv"))
    with open(os.path.join(out, f"bench_{a.tag}.json")) as fh:
        line = [ln for ln in fh if ln.startswith("{")][-1]
    with open(os.path.join(prof, f"{a.tag}_bench.json"), "w") as fh:
        fh.write(line)
    pmc_path = os.path.join(out, f"pmc_{a.tag}", "summary.json")
    if os.path.exists(pmc_path):
        with open(pmc_path) as fh:
            pmc = json.load(fh)
        with open(os.path.join(prof, f"{a.tag}_pmc.json"), "w") as fh:
            json.dump(pmc, fh, indent=1)
        traffic = {short(k): {"config": a.config, "hbm_bytes_per_launch": int(v["HBM_BYTES_CORRECTED"]),
                              "fetch_kib": v["FETCH_SIZE"], "write_kib": v["WRITE_SIZE"], "source": f"{a.tag}_pmc.json"}
                   for k, v in pmc.items() if "HBM_BYTES_CORRECTED" in v}
        with open(os.path.join(prof, "pmc_traffic.json"), "w") as fh:
            json.dump(traffic, fh, indent=1)
    print(sorted(os.listdir(prof)))


if __name__ == "__main__":
    main()
