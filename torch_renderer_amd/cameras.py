"""Cameras (subset of upstream pytorch3d/renderer/cameras.py used by the reference).

Every camera reduces, per view, to the record consumed by the kernels
(include/mi355r.h ``mr_view_t``): R, T in PyTorch3D's row-vector convention and
the NDC affine (ax, bx, ay, by) such that
    ndc_x = ax * X_view/Z_view + bx,  ndc_y = ay * Y_view/Z_view + by.
"""
from __future__ import annotations

import math

import torch


def _as_batch(x, n_cols, device, default):
    if x is None:
        x = default
    t = torch.as_tensor(x, dtype=torch.float32, device=device)
    return t.reshape(-1, n_cols) if n_cols else t.reshape(-1)


class CamerasBase:
    def __init__(self, R=None, T=None, device="cpu"):
        self.device = torch.device(device)
        R = torch.eye(3, device=self.device)[None] if R is None else torch.as_tensor(R, device=self.device)
        T = torch.zeros(1, 3, device=self.device) if T is None else torch.as_tensor(T, device=self.device)
        self.R = R.float().reshape(-1, 3, 3)
        self.T = T.float().reshape(-1, 3)

    def __setattr__(self, k, v):
        # every attribute assignment bumps the generation _param_key keys on (the scalar attributes and the
        # set of tensor attributes change only through here; in-place tensor edits are seen by their versions)
        d = self.__dict__
        d["_attr_gen"] = d.get("_attr_gen", 0) + 1
        object.__setattr__(self, k, v)

    def __delattr__(self, k):
        d = self.__dict__
        d["_attr_gen"] = d.get("_attr_gen", 0) + 1
        object.__delattr__(self, k)

    def __len__(self):
        return max(self.R.shape[0], self.T.shape[0], getattr(self, "_n_intr", 1))

    def is_perspective(self):
        return True

    def get_znear(self):
        return getattr(self, "znear", None)

    def get_camera_center(self, **kwargs):
        """World-space centre from the camera's R, T (kwargs R/T override)."""
        R = kwargs.get("R", self.R).reshape(-1, 3, 3)
        T = kwargs.get("T", self.T).reshape(-1, 3)
        # X_view = X @ R + T = 0  =>  X = -T @ R^T
        return -torch.bmm(T[:, None, :], R.transpose(1, 2))[:, 0, :]

    def ndc_affine(self, image_size):  # (N,4): ax, bx, ay, by
        raise NotImplementedError

    def __getitem__(self, i):
        """Camera i of the batch (mesh_deformer.py:197 renders with ``target_cameras[j]``): every
        per-camera tensor attribute with a batch dimension > 1 is sliced, singletons broadcast."""
        import copy

        n = len(self)
        if not -n <= i < n:
            raise IndexError(f"camera index {i} out of range for a batch of {n}")
        if i < 0:  # cams[-1] is the last camera (a slice v[-1:0] would be empty)
            i += n
        c = copy.copy(self)
        c.__dict__ = {k: v for k, v in self.__dict__.items() if not k.startswith("_") or k in ("_in_ndc",)}
        for k, v in list(c.__dict__.items()):
            if torch.is_tensor(v) and v.dim() >= 1 and v.shape[0] == n and n > 1 and k != "image_size":
                c.__dict__[k] = v[i:i + 1]
        if hasattr(self, "_n_intr"):
            c._n_intr = 1 if self._n_intr > 1 else self._n_intr
        return c

    def to(self, device):
        self.device = torch.device(device)
        for k, v in list(self.__dict__.items()):
            if torch.is_tensor(v):
                setattr(self, k, v.to(self.device))
        return self


class PerspectiveCameras(CamerasBase):
    """focal_length / principal_point in pixels when in_ndc=False (torch_renderer.py:61-71),
    or an explicit 4x4 K (renderer.py:47-50,69)."""

    def __init__(self, focal_length=1.0, principal_point=((0.0, 0.0),), R=None, T=None, K=None, device="cpu",
                 in_ndc=True, image_size=None):
        super().__init__(R, T, device)
        self._in_ndc = bool(in_ndc)
        if K is not None:
            K = torch.as_tensor(K, dtype=torch.float32, device=self.device).reshape(-1, 4, 4)
            fx, fy, px, py = K[:, 0, 0], K[:, 1, 1], K[:, 0, 2], K[:, 1, 2]
        else:
            fl = torch.as_tensor(focal_length, dtype=torch.float32, device=self.device)
            fl = fl.reshape(-1, 1).expand(-1, 2) if fl.dim() < 2 or fl.shape[-1] == 1 else fl.reshape(-1, 2)
            pp = _as_batch(principal_point, 2, self.device, ((0.0, 0.0),))
            fx, fy = fl[:, 0], fl[:, 1]
            px, py = pp[:, 0], pp[:, 1]
        self.fx, self.fy, self.px, self.py = fx, fy, px, py
        self._n_intr = fx.shape[0]
        self.image_size = None if image_size is None else torch.as_tensor(image_size).reshape(-1, 2)
        if not self._in_ndc and self.image_size is None:
            raise ValueError("PerspectiveCameras(in_ndc=False) needs image_size")

    def in_ndc(self):
        return self._in_ndc

    def ndc_affine(self, image_size):
        H, W = image_size
        if self._in_ndc:
            return torch.stack([self.fx, self.px, self.fy, self.py], dim=1)
        hw = self.image_size.to(self.fx.device).float()
        Hc, Wc = hw[:, 0], hw[:, 1]
        s = torch.minimum(Hc, Wc) / 2.0
        ax = self.fx.double() / s.double()
        bx = (Wc.double() / 2.0 - self.px.double()) / s.double()
        ay = self.fy.double() / s.double()
        by = (Hc.double() / 2.0 - self.py.double()) / s.double()
        return torch.stack([ax, bx, ay, by], dim=1).float()


class FoVPerspectiveCameras(CamerasBase):
    """OpenGL-style perspective camera (camera_pose_optimizer.py:105)."""

    def __init__(self, znear=1.0, zfar=100.0, aspect_ratio=1.0, fov=60.0, degrees=True, R=None, T=None,
                 device="cpu"):
        super().__init__(R, T, device)
        self.znear, self.zfar = float(znear), float(zfar)
        self.aspect_ratio, self.fov, self.degrees = float(aspect_ratio), float(fov), bool(degrees)

    def ndc_affine(self, image_size):
        fov = math.radians(self.fov) if self.degrees else self.fov
        t = math.tan(fov / 2.0)
        ax = 1.0 / (t * self.aspect_ratio)
        ay = 1.0 / t
        n = max(self.R.shape[0], self.T.shape[0])
        return torch.tensor([[ax, 0.0, ay, 0.0]], dtype=torch.float32, device=self.device).expand(n, 4).contiguous()


def _param_key(cameras):
    """The caches' key: the camera's attribute generation (CamerasBase.__setattr__ bumps it on every
    assignment, so it covers the scalar attributes — FoV cameras keep fov / aspect_ratio / znear as floats —
    and which tensors are attached) and (storage, version) of its tensor attributes (in-place edits). The
    tensor attribute names are listed once per generation (an eager loop calls this on every render)."""
    d = cameras.__dict__
    gen = d.get("_attr_gen", 0)
    names = d.get("_pk_names")
    if names is None or names[0] != gen:
        names = (gen, tuple(k for k in sorted(d) if (not k.startswith("_") or k == "_in_ndc") and torch.is_tensor(d[k])))
        d["_pk_names"] = names
    out = [gen]
    for k in names[1]:
        v = d[k]
        out.append(v.data_ptr())
        out.append(v._version)
    return tuple(out)


def cached_ndc_affine(cameras: CamerasBase, image_size, device):
    """ndc_affine on `device`, recomputed only when the camera's tensors change (their
    storage or version) — the per-call double-precision conversions are host-side launches."""
    key = (int(image_size[0]), int(image_size[1]), device, _param_key(cameras))
    c = cameras.__dict__.get("_ndc_cache")
    if c is None or c[0] != key:
        c = (key, cameras.ndc_affine(image_size).to(device).contiguous())
        cameras.__dict__["_ndc_cache"] = c
    return c[1]


def cached_camera_center(cameras: CamerasBase, device):
    """get_camera_center() (camera's own R, T) on `device`, cached like cached_ndc_affine."""
    key = (device, _param_key(cameras))
    c = cameras.__dict__.get("_cc_cache")
    if c is None or c[0] != key:
        c = (key, cameras.get_camera_center().to(device).contiguous())
        cameras.__dict__["_cc_cache"] = c
    return c[1]


def view_batch(cameras: CamerasBase, image_size, R=None, T=None, n_views=None):
    """(R (N,3,3), T (N,3), intr (N,4)) for N views, broadcasting singleton camera params."""
    R = cameras.R if R is None else R
    T = cameras.T if T is None else T
    R = R.reshape(-1, 3, 3)
    T = T.reshape(-1, 3)
    intr = cached_ndc_affine(cameras, image_size, R.device)
    N = n_views or max(R.shape[0], T.shape[0], intr.shape[0])
    for name, t in (("R", R), ("T", T), ("intrinsics", intr)):
        if t.shape[0] not in (1, N):
            raise ValueError(f"camera {name} batch {t.shape[0]} does not broadcast to {N} views")
    return R.expand(N, 3, 3), T.expand(N, 3), intr.expand(N, 4)
