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
