"""Experiment builds of libmi355r.so with extra -D flags into exp/ (run with MI355R_LIB=exp/<name>.so).
python tools/build_variant.py NAME -DFOO -DBAR=2 ..."""
import os
import subprocess
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from torch_renderer_amd import _build  # noqa: E402

name, defs = sys.argv[1], sys.argv[2:]
out = os.path.join(_build._HERE, "..", "exp", name + ".so")
os.makedirs(os.path.dirname(out), exist_ok=True)
subprocess.run([_build.hipcc(), *_build.HIPCC_FLAGS, *defs, "-o", out, *_build.sources()], check=True)
print(out)
