"""Round-6 host-side checks (no GPU): the C++ autograd glue reports the torch it was built against and loads
only into that torch (a torch upgrade must not leave a stale _mr_torch.so that fails later); the
fixed-point cutoff the backward uses is the documented one."""
import os
import re

import torch

from torch_renderer_amd import _build, _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_torch_ext_reports_its_torch():
    mod = _lib.torch_ext()
    assert mod.built_with_torch == torch.__version__
    assert bool(mod.built_with_cxx11_abi) == bool(torch._C._GLIBCXX_USE_CXX11_ABI)


def test_torch_ext_stamp_drives_the_rebuild():
    with open(_build.TORCH_EXT_STAMP) as fh:
        assert fh.read().strip() == _build.torch_stamp()
    assert not _build.torch_ext_needs_build()


def test_fixed_point_cutoff_is_2_pow_24():
    src = open(os.path.join(ROOT, "torch_renderer_amd", "csrc", "mr_common.h")).read()
    m = re.search(r"#define MR_FIX_MAX ([0-9.]+)f", src)
    assert m and float(m.group(1)) == 2.0 ** 24
