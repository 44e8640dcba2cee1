"""Rotation helpers used by the reference callers (pytorch3d.transforms /
pytorch3d.renderer.cameras look-at utilities): quaternion_to_matrix
(camera_pose_optimizer.py:241), matrix_to_quaternion (:170),
look_at_view_transform (:167), plus an OpenCV look-at used by the benchmark.
Formulas restate upstream pytorch3d/transforms/rotation_conversions.py and
pytorch3d/renderer/cameras.py."""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def quaternion_to_matrix(quaternions: torch.Tensor) -> torch.Tensor:
    """Real-part-first quaternions (not renormalised: two_s = 2/|q|^2) -> rotation matrices
    (upstream pytorch3d.transforms.quaternion_to_matrix). HIP float32 tensors take one launch each way
    (mr_quaternion_to_matrix[_backward], torch's elementwise operation order) through the C++ autograd node
    _mr_torch.quaternion_to_matrix — instead of ~30 tiny torch kernels forward and ~60 backward per optimiser
    step (camera_pose_optimizer.py:241); others (the CPU oracle) the torch formula."""
    if quaternions.is_cuda and quaternions.dtype == torch.float32 and quaternions.shape[-1] == 4:
        from . import _lib

        return _lib.torch_ext().quaternion_to_matrix(quaternions)
    return quaternion_to_matrix_torch(quaternions)


def quaternion_to_matrix_torch(quaternions: torch.Tensor) -> torch.Tensor:
    """The torch formula of upstream quaternion_to_matrix (any device / dtype)."""
    r, i, j, k = torch.unbind(quaternions, -1)
    two_s = 2.0 / (quaternions * quaternions).sum(-1)
    o = torch.stack((
        1 - two_s * (j * j + k * k), two_s * (i * j - k * r), two_s * (i * k + j * r),
        two_s * (i * j + k * r), 1 - two_s * (i * i + k * k), two_s * (j * k - i * r),
        two_s * (i * k - j * r), two_s * (j * k + i * r), 1 - two_s * (i * i + j * j),
    ), -1)
    return o.reshape(quaternions.shape[:-1] + (3, 3))


def _sqrt_positive_part(x: torch.Tensor) -> torch.Tensor:
    ret = torch.zeros_like(x)
    pos = x > 0
    ret[pos] = torch.sqrt(x[pos])
    return ret


def matrix_to_quaternion(matrix: torch.Tensor) -> torch.Tensor:
    if matrix.size(-1) != 3 or matrix.size(-2) != 3:
        raise ValueError(f"Invalid rotation matrix shape {matrix.shape}.")
    batch_dim = matrix.shape[:-2]
    m00, m01, m02, m10, m11, m12, m20, m21, m22 = torch.unbind(matrix.reshape(batch_dim + (9,)), dim=-1)
    q_abs = _sqrt_positive_part(torch.stack([1.0 + m00 + m11 + m22, 1.0 + m00 - m11 - m22,
                                             1.0 - m00 + m11 - m22, 1.0 - m00 - m11 + m22], dim=-1))
    quat_by_rijk = torch.stack([
        torch.stack([q_abs[..., 0] ** 2, m21 - m12, m02 - m20, m10 - m01], dim=-1),
        torch.stack([m21 - m12, q_abs[..., 1] ** 2, m10 + m01, m02 + m20], dim=-1),
        torch.stack([m02 - m20, m10 + m01, q_abs[..., 2] ** 2, m12 + m21], dim=-1),
        torch.stack([m10 - m01, m20 + m02, m21 + m12, q_abs[..., 3] ** 2], dim=-1),
    ], dim=-2)
    flr = torch.tensor(0.1).to(dtype=q_abs.dtype, device=q_abs.device)
    quat_candidates = quat_by_rijk / (2.0 * q_abs[..., None].max(flr))
    out = quat_candidates[F.one_hot(q_abs.argmax(dim=-1), num_classes=4) > 0.5, :].reshape(batch_dim + (4,))
    return out


def camera_position_from_spherical_angles(distance, elevation, azimuth, degrees=True, device="cpu"):
    d, e, a = torch.broadcast_tensors(*(torch.as_tensor(x, dtype=torch.float32, device=device)
                                        for x in (distance, elevation, azimuth)))
    if degrees:
        e = math.pi / 180.0 * e
        a = math.pi / 180.0 * a
    x = d * torch.cos(e) * torch.sin(a)
    y = d * torch.sin(e)
    z = d * torch.cos(e) * torch.cos(a)
    return torch.stack([x, y, z], dim=-1).view(-1, 3)


def look_at_rotation(camera_position, at=((0, 0, 0),), up=((0, 1, 0),), device="cpu"):
    camera_position = torch.as_tensor(camera_position, dtype=torch.float32, device=device).view(-1, 3)
    at = torch.as_tensor(at, dtype=torch.float32, device=device).view(-1, 3)
    up = torch.as_tensor(up, dtype=torch.float32, device=device).view(-1, 3)
    camera_position, at, up = torch.broadcast_tensors(camera_position, at, up)
    z_axis = F.normalize(at - camera_position, eps=1e-5)
    x_axis = F.normalize(torch.cross(up, z_axis, dim=1), eps=1e-5)
    y_axis = F.normalize(torch.cross(z_axis, x_axis, dim=1), eps=1e-5)
    is_close = torch.isclose(x_axis, torch.tensor(0.0, device=x_axis.device), atol=5e-3).all(dim=1, keepdim=True)
    if is_close.any():
        replacement = F.normalize(torch.cross(y_axis, z_axis, dim=1), eps=1e-5)
        x_axis = torch.where(is_close, replacement, x_axis)
    R = torch.cat((x_axis[:, None, :], y_axis[:, None, :], z_axis[:, None, :]), dim=1)
    return R.transpose(1, 2)


def look_at_view_transform(dist=1.0, elev=0.0, azim=0.0, degrees=True, eye=None, at=((0, 0, 0),),
                           up=((0, 1, 0),), device="cpu"):
    """PyTorch3D convention (X_view = X_world @ R + T)."""
    if eye is not None:
        C = torch.as_tensor(eye, dtype=torch.float32, device=device).view(-1, 3)
    else:
        C = camera_position_from_spherical_angles(dist, elev, azim, degrees=degrees, device=device)
        C = C + torch.as_tensor(at, dtype=torch.float32, device=device).view(-1, 3)
    R = look_at_rotation(C, at, up, device=device)
    T = -torch.bmm(R.transpose(1, 2), C[:, :, None])[:, :, 0]
    return R, T


def opencv_look_at(centers, targets, up=(0.0, 1.0, 0.0)):
    """OpenCV world->camera (R, t): camera at `centers` looking at `targets`
    (x right, y down, z forward): X_cam = R @ X_world + t."""
    centers = torch.as_tensor(centers, dtype=torch.float64).view(-1, 3)
    targets = torch.as_tensor(targets, dtype=torch.float64).view(-1, 3).expand_as(centers)
    up = torch.as_tensor(up, dtype=torch.float64).view(1, 3).expand_as(centers)
    z = F.normalize(targets - centers, dim=1)
    x = F.normalize(torch.cross(z, up, dim=1), dim=1)
    y = torch.cross(z, x, dim=1)
    R = torch.stack([x, y, z], dim=1)
    t = -(R @ centers[:, :, None])[:, :, 0]
    return R.float(), t.float()


_SIGN_CACHE: dict = {}


def _col_sign(device, dtype):
    key = (str(device), dtype)
    s = _SIGN_CACHE.get(key)
    if s is None:
        s = _SIGN_CACHE[key] = torch.tensor([-1.0, -1.0, 1.0], dtype=dtype, device=device)
    return s


def opencv_to_pytorch3d(R: torch.Tensor, tvec: torch.Tensor):
    """DifferentiableRenderer._camera_pose_from_opencv_to_pytorch (torch_renderer.py:73-80):
    R_p = R^T with columns 0 and 1 negated, T_p = tvec with entries 0 and 1 negated.
    One multiply each (exact: x * -1), no in-place slice updates in the autograd graph."""
    s = _col_sign(R.device, R.dtype)
    return R.transpose(1, 2) * s, tvec * s.to(tvec.dtype)
