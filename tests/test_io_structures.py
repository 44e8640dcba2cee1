"""OBJ/MTL loading (pytorch3d.io semantics), bundled assets, Meshes / textures, cameras and
rotation helpers — all CPU."""
import math
import os

import numpy as np
import pytest
import torch

from torch_renderer_amd import (FoVPerspectiveCameras, Meshes, PerspectiveCameras, TexturesUV, TexturesVertex,
                                load_obj, load_objs_as_meshes, look_at_view_transform, matrix_to_quaternion,
                                quaternion_to_matrix)
from torch_renderer_amd.assets import load_asset, load_asset_arrays
from torch_renderer_amd.cameras import view_batch
from torch_renderer_amd.transforms import opencv_look_at, opencv_to_pytorch3d

REF = "/root/reference/data"

OBJ = """# test
mtllib m.mtl
v 0 0 0
v 1 0 0
v 1 1 0
v 0 1 0
v 0.5 0.5 1
vt 0 0
vt 1 0
vt 1 1
vt 0 1
vn 0 0 1
usemtl mat0
f 1/1/1 2/2/1 3/3/1 4/4/1
f -1 -4 -3
"""
MTL = "newmtl mat0\nKd 0.5 0.5 0.5\nmap_Kd tex.png\n"


def test_load_obj_fan_triangulation_negative_indices(tmp_path):
    (tmp_path / "m.obj").write_text(OBJ)
    (tmp_path / "m.mtl").write_text(MTL)
    from PIL import Image

    Image.fromarray(np.arange(4 * 4 * 3, dtype=np.uint8).reshape(4, 4, 3)).save(tmp_path / "tex.png")
    verts, faces, aux = load_obj(tmp_path / "m.obj")
    assert verts.shape == (5, 3)
    assert faces.verts_idx.tolist() == [[0, 1, 2], [0, 2, 3], [4, 1, 2]]
    assert faces.textures_idx.tolist() == [[0, 1, 2], [0, 2, 3], [-1, -1, -1]]
    assert aux.verts_uvs.shape == (4, 2)
    img = aux.texture_images["mat0"]
    assert img.dtype == torch.float32 and img.shape == (4, 4, 3)
    assert torch.equal(img, torch.from_numpy(np.arange(48, dtype=np.uint8).reshape(4, 4, 3).astype(np.float32) / 255.0))
    m = load_objs_as_meshes([tmp_path / "m.obj"])
    assert isinstance(m.textures, TexturesUV) and len(m) == 1


def test_missing_texture_gives_untextured_mesh(tmp_path):
    (tmp_path / "m.obj").write_text(OBJ)
    (tmp_path / "m.mtl").write_text("newmtl mat0\nmap_Kd /definitely/missing.png\n")
    m = load_objs_as_meshes([tmp_path / "m.obj"])
    assert m.textures is None


@pytest.mark.parametrize("name,V,F", [("cow", 2930, 5856), ("teapot", 1292, 2464), ("sphere", 2562, 5120),
                                      ("dolphin", 2562, 5120)])
def test_assets(name, V, F):
    d = load_asset_arrays(name)
    assert d["verts"].shape == (V, 3) and d["faces"].shape == (F, 3)
    m = load_asset(name)
    assert m.shared_faces().shape == (F, 3)
    if name == "cow":
        assert m.textures.maps_list()[0].shape == (1024, 1024, 3)


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference data not present")
def test_assets_match_reference_objs():
    for name, rel in (("cow", "cow_mesh/cow.obj"), ("teapot", "teapot.obj")):
        v, f, aux = load_obj(os.path.join(REF, rel))
        d = load_asset_arrays(name)
        assert np.array_equal(v.numpy(), d["verts"]) and np.array_equal(f.verts_idx.numpy(), d["faces"])


def test_meshes_extend_is_shared_and_packs_like_pytorch3d():
    v = torch.rand(5, 3)
    f = torch.tensor([[0, 1, 2], [2, 3, 4]])
    m = Meshes([v], [f], TexturesVertex([torch.rand(5, 3)])).extend(3)
    assert len(m) == 3 and m.is_shared()
    assert m.verts_packed().shape == (15, 3)
    fp = m.faces_packed()
    assert fp.tolist()[2:4] == [[5, 6, 7], [7, 8, 9]]
    assert m.mesh_to_faces_packed_first_idx().tolist() == [0, 2, 4]
    assert m.verts_padded().shape == (3, 5, 3)
    m2 = Meshes([v, v + 1], [f, f])
    assert not m2.is_shared() and len(m2.extend(2)) == 4
    off = m.offset_verts(torch.ones(15, 3))
    assert torch.allclose(off.verts_list()[1], v + 1)


def test_quaternion_roundtrip_and_lookat():
    q = torch.tensor([[0.9, 0.1, -0.3, 0.2]])
    q = q / q.norm()
    R = quaternion_to_matrix(q)
    assert torch.allclose(R @ R.transpose(1, 2), torch.eye(3)[None], atol=1e-6)
    q2 = matrix_to_quaternion(R)
    assert torch.allclose(q2, q, atol=1e-6) or torch.allclose(q2, -q, atol=1e-6)
    R, T = look_at_view_transform(0.7, 30, 60)
    # camera centre C = -T R^T sits at distance 0.7 from the origin it looks at
    C = -(T[:, None, :] @ R.transpose(1, 2))[:, 0]
    assert math.isclose(C.norm().item(), 0.7, rel_tol=1e-5)
    # the origin projects to the image centre (view x = y = 0)
    v = torch.zeros(1, 3) @ R[0] + T[0]
    assert abs(v[0, 0]) < 1e-6 and abs(v[0, 1]) < 1e-6 and v[0, 2] > 0


def test_perspective_camera_screen_convention():
    """in_ndc=False: a point at OpenCV pixel (u, v) = (xi + 0.5, yi + 0.5) lands on the
    NDC centre of output pixel (xi, yi) (torch_renderer.py:61-80)."""
    H, W = 60, 80
    fx, fy, px, py = 70.0, 65.0, 41.0, 28.5
    K = torch.tensor([[fx, 0, px], [0, fy, py], [0, 0, 1.0]])
    cam = PerspectiveCameras(focal_length=torch.tensor([[fx, fy]]), principal_point=torch.tensor([[px, py]]),
                             in_ndc=False, image_size=torch.tensor([[H, W]]))
    R_cv = torch.eye(3)[None]
    t_cv = torch.zeros(1, 3)
    Rp, Tp = opencv_to_pytorch3d(R_cv, t_cv)
    _, _, intr = view_batch(cam, (H, W), Rp, Tp)
    ax, bx, ay, by = intr[0].tolist()
    xi, yi, Z = 13, 41, 2.0
    Xc = torch.tensor([(xi + 0.5 - px) / fx * Z, (yi + 0.5 - py) / fy * Z, Z])  # OpenCV camera frame
    Xv = Xc @ Rp[0] + Tp[0]
    ndc = (ax * Xv[0] / Xv[2] + bx, ay * Xv[1] / Xv[2] + by)
    from oracle.spec_np import pix_to_ndc

    assert math.isclose(ndc[0], pix_to_ndc(W - 1 - xi, W, H), abs_tol=1e-5)
    assert math.isclose(ndc[1], pix_to_ndc(H - 1 - yi, H, W), abs_tol=1e-5)
    del K


def test_fov_camera_and_opencv_lookat():
    cam = FoVPerspectiveCameras(fov=60.0)
    ax, bx, ay, by = cam.ndc_affine((64, 64))[0].tolist()
    assert math.isclose(ax, 1 / math.tan(math.radians(30)), rel_tol=1e-6) and bx == 0 and by == 0
    R, t = opencv_look_at(torch.tensor([[0.0, 0.0, -2.0]]), torch.zeros(1, 3))
    Xc = R[0] @ torch.zeros(3) + t[0]
    assert torch.allclose(Xc, torch.tensor([0.0, 0.0, 2.0]), atol=1e-6)
