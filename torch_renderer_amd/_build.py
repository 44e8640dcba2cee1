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
    if force or needs_build():
        cmd = [hipcc(), *HIPCC_FLAGS, "-o", OUT + ".tmp", *sources()]
        if verbose:
            print("[mi355r] " + " ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(OUT + ".tmp", OUT)
    build_torch_ext(force=force, verbose=verbose)
    return OUT


# The fused render's autograd node in C++ (csrc/mr_torch.cpp, host code only): compiled with the host
# compiler against torch's headers and libraries, in-tree like libmi355r.so (it travels with the tree).
TORCH_EXT = os.path.join(_HERE, "_mr_torch.so")
TORCH_EXT_SRC = os.path.join(CSRC, "mr_torch.cpp")


def torch_ext_cmd(out: str):
    import sysconfig

    import torch
    from torch.utils import cpp_extension as ce

    tdir = os.path.dirname(torch.__file__)
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    cxx = os.environ.get("CXX", "g++")
    incs = [f"-I{p}" for p in ce.include_paths()] + [f"-I{sysconfig.get_paths()['include']}",
                                                     f"-I{os.path.join(rocm, 'include')}",
                                                     f"-I{os.path.join(_HERE, '..', 'include')}"]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return [cxx, "-O2", "-std=c++17", "-fPIC", "-shared", "-DTORCH_EXTENSION_NAME=_mr_torch",
            f'-DMR_TORCH_VERSION="{torch.__version__}"',
            "-DTORCH_API_INCLUDE_EXTENSION_H", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DUSE_ROCM",
            "-D__HIP_PLATFORM_AMD__=1", *incs, TORCH_EXT_SRC, "-o", out,
            f"-L{os.path.join(tdir, 'lib')}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_python",
            f"-Wl,-rpath,{os.path.join(tdir, 'lib')}"]


TORCH_EXT_STAMP = TORCH_EXT + ".stamp"  # the torch version and C++ ABI flag the extension was built against


def torch_stamp() -> str:
    import torch

    return f"{torch.__version__} cxx11_abi={int(torch._C._GLIBCXX_USE_CXX11_ABI)}"


def torch_ext_needs_build() -> bool:
    if not os.path.exists(TORCH_EXT):
        return True
    t = os.path.getmtime(TORCH_EXT)
    deps = [TORCH_EXT_SRC, os.path.join(_HERE, "..", "include", "mi355r.h"), os.path.abspath(__file__)]
    if any(os.path.getmtime(d) > t for d in deps if os.path.exists(d)):
        return True
    try:  # a torch upgrade (or another ABI) leaves the sources older than the .so: rebuild on the stamp
        with open(TORCH_EXT_STAMP) as fh:
            return fh.read().strip() != torch_stamp()
    except OSError:
        return True


def build_torch_ext(force: bool = False, verbose: bool = True) -> str:
    if not force and not torch_ext_needs_build():
        return TORCH_EXT
    cmd = torch_ext_cmd(TORCH_EXT + ".tmp")
    if verbose:
        print("[mi355r] " + " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(TORCH_EXT + ".tmp", TORCH_EXT)
    with open(TORCH_EXT_STAMP, "w") as fh:
        fh.write(torch_stamp() + "\n")
    return TORCH_EXT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
