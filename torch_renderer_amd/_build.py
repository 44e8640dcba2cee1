"""Build ``libmi355r.so`` in-tree with hipcc for gfx950 (cross-compiles without a GPU).

    python -m torch_renderer_amd._build
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(_HERE, "csrc")
OUT = os.path.join(_HERE, "libmi355r.so")

HIPCC_FLAGS = [
    "--offload-arch=gfx950",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-shared",
    # Bit-exact integer outputs need the CPU operand order: no FMA contraction.
    "-ffp-contract=off",
    # No SLP (straight-line) vectorisation into v_pk_* pairs: the pairs need operand copies into
    # adjacent registers, which cost more than they save. k_bwd_fused: 239 -> 194 VGPRs, 505 -> 247
    # v_mov, 88.5 -> 82.6 us (profiles/r2k_noslp_ab.txt).
    "-fno-slp-vectorize",
    # Machine scheduler biased to ILP over occupancy: each wave of the latency-bound kernels hides
    # more of its own latency. k_bwd_fused 82.9 -> 79.8 us, k_tile_raster 85.8 -> 83.8 us
    # (max-memory-clause: no change; profiles/r2l_sched_ab.txt).
    "-mllvm",
    "-amdgpu-sched-strategy=max-ilp",
]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required)")


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def needs_build(out: str = OUT) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    deps = sources() + glob.glob(os.path.join(CSRC, "*.h")) + [os.path.join(_HERE, "..", "include", "mi355r.h")]
    deps.append(os.path.abspath(__file__))  # compiler flags live here
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = True) -> str:
    if not force and not needs_build():
        return OUT
    cmd = [hipcc(), *HIPCC_FLAGS, "-o", OUT + ".tmp", *sources()]
    if verbose:
        print("[mi355r] " + " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
