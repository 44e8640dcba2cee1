"""PMC summary (tools/pmc_summary.py's summary.json of one build) -> profiles/pmc_traffic.json, the per-launch HBM
bytes bench.py reports as roofline.traffic: FETCH_SIZE x 2 + WRITE_SIZE (KiB), the gfx950 correction of
MI355X_MICROARCH.md §HBM (calibrated on this workload: 99.5 % of the memory-side read requests are 128 B,
profiles/r5z_pmc_reqsize.json). Keys are bench.py's kernel names (the HIP-event timer's).
python tools/pmc_traffic.py gpurun_out/pmc_TAG/summary.json SOURCE_NAME [config]"""
import json
import os
import re
import sys

# rocprof kernel name (template arguments stripped) -> bench.py / _lib.timing_read name
NAMES = {"k_bin_rect_world": "k_bin_rect", "k_bin_view": "k_bin_view", "k_tile_raster": "k_tile_raster",
         "k_shade": "k_shade<1>", "k_shade_render": "k_shade<1>", "k_bwd_fused": "k_bwd_fused",
         "k_rt_vgrad_a": "k_rt_vgrad_a", "k_vgrad_b": "k_vgrad_b", "k_unit_order": "k_unit_order"}


def main(path, source, config="cow-512x512-64"):
    d = json.load(open(path))
    out = {}
    for k, c in d.items():
        base = re.sub(r"^void ", "", k).split("<")[0].strip()
        name = NAMES.get(base)
        if name is None or "FETCH_SIZE" not in c or "WRITE_SIZE" not in c:
            continue
        out[name] = {"config": config, "hbm_bytes_per_launch": int(round((2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024)),
                     "fetch_kib": c["FETCH_SIZE"], "write_kib": c["WRITE_SIZE"], "source": source, "rocprof_name": k,
                     "valu_insts_per_launch": c.get("SQ_INSTS_VALU"),
                     "note": "FETCH_SIZE x2 (calibrated: 99.5 % of the memory-side read requests are 128 B, "
                             "r5z_pmc_reqsize.json) + WRITE_SIZE"}
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "pmc_traffic.json")
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps({k: v["hbm_bytes_per_launch"] for k, v in out.items()}))


if __name__ == "__main__":
    main(*sys.argv[1:])
