"""Round-5 host-side checks (CPU, no GPU): the distinct-mesh union topology cache and the reshade
entry's lifetime rules."""
import torch

from torch_renderer_amd import torch_renderer as TR
from torch_renderer_amd.structures import Meshes


def _tet(shift):
    v = torch.tensor([[0.0, 0, 0], [1, 0, 0], [0, 1, 0], [0, 0, 1]]) + shift
    f = torch.tensor([[0, 1, 2], [0, 1, 3], [0, 2, 3], [1, 2, 3]])
    return v, f


def test_union_topology_survives_vertex_updates():
    """the union depends on faces and vertex counts only. An in-place vertex update (an
    optimiser step) keeps the cached union faces tensor (same object: its CSR stays cached); an in-place
    faces edit rebuilds it."""
    (v1, f1), (v2, f2) = _tet(0.0), _tet(2.0)
    v1.requires_grad_(True)
    m = Meshes([v1, v2], [f1, f2])
    u1 = TR._union_topology(m)
    with torch.no_grad():
        v1.add_(0.5)  # version bump of the verts
    u2 = TR._union_topology(m)
    assert u2[0] is u1[0]
    assert torch.equal(u1[0], torch.cat([f1, f2 + 4]))
    assert u1[1].tolist() == [0, 4, 8] and u1[2].tolist() == [4, 4] and u1[4].tolist() == [0, 4, 8]
    f2[0, 0] = 1  # in-place faces edit
    u3 = TR._union_topology(m)
    assert u3[0] is not u1[0] and int(u3[0][4, 0]) == 5


def test_parity_summary_parses_report_lines(tmp_path, capsys):
    """tools/parity_summary.py (the committed profiles/*_parity_summary.txt): every report() line form — with the
    float64 shadow's ratios, with the ill-conditioned count only, and the plain form — is parsed, and the worst
    err/limit is found."""
    import importlib.util
    import os

    spec = importlib.util.spec_from_file_location(
        "parity_summary", os.path.join(os.path.dirname(__file__), "..", "tools", "parity_summary.py"))
    ps = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ps)
    log = tmp_path / "p.log"
    log.write_text(
        "tests/test_gpu_configs.py::test_a [parity] A depth: n = 10, max|err| = 0.000e+00, scale = 1.0e+00, "
        "worst err/limit = 0.000, ill-conditioned = 0, vs f64: GPU 0.011 / f32 oracle 0.012 of the bar at (0,) "
        "(got 0, ref 0)\n"
        "[parity] A grad: n = 7, max|err| = 1e-3, scale = 2.0e+00, worst err/limit = 0.628, ill-conditioned = 3 at (1,)"
        " (got 1, ref 1)\n"
        "tests/test_gpu_configs.py::test_b [parity] B loss: n = 1, max|err| = 0.0, scale = 1.0, worst err/limit = 0.100"
        " at () (got 1, ref 1)\n"
        "[parity] pose_loss total: 0.5 vs torch 0.5\n")
    ps.main(str(log))
    out = capsys.readouterr().out
    assert out.startswith("3 [parity] lines")
    assert "worst err/limit over all lines: 0.628 (test_a: A grad)" in out
    assert "0.011" in out and "0.012" in out
