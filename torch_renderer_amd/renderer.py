"""Drop-in for the reference's ``renderer.py`` ``Renderer`` class (renderer.py:34-101).

Same constructor (fixed intrinsics/extrinsic of the reference's RealSense setup, 4x4
screen-space K, PointLights at (0, 0, -3)), ``load_meshes``, ``update_light_position``,
``build_color_renderer`` and ``render() -> (N, H, W, 4)`` RGBA, backed by the fused MI355X
render (one launch per call; camera centre for specular from the camera's own R, T as in
upstream SoftPhongShader). The reference's module-level demo on a machine-specific path
(renderer.py:105-114) is not reproduced.
"""
from __future__ import annotations

import numpy as np
import torch

from .cameras import PerspectiveCameras
from .io import load_objs_as_meshes
from .mesh_renderer import MeshRasterizer, MeshRenderer, PointLights, RasterizationSettings, SoftPhongShader

# renderer.py:46-58
_K = [[914.4831543, 0.0, 645.47546387, 0.0],
      [0.0, 913.00628662, 367.93243408, 0.0],
      [0.0, 0.0, 0.0, 1.0],
      [0.0, 0.0, 1.0, 0.0]]
_EXTRINSIC = np.array([[-0.91087912, -0.40173757, -0.09437244, 0.1],
                       [-0.13151312, 0.49935385, -0.85635859, 0.1],
                       [0.39115666, -0.76762794, -0.50768475, 0.374397],
                       [0.0, 0.0, 0.0, 1.0]])


class Renderer:
    def __init__(self, image_size=(720, 1280)):
        if torch.cuda.is_available():
            self.device = torch.device("cuda:0")
            torch.cuda.set_device(self.device)
        else:
            self.device = torch.device("cpu")  # as the reference; rendering then raises (no CPU fallback)
        self.image_size = image_size
        K = torch.tensor([_K], device=self.device)
        camera_pose = _EXTRINSIC
        R = torch.tensor(np.array([camera_pose[:3, :3]]), device=self.device)
        t = torch.tensor(np.array([camera_pose[:3, 3]]), device=self.device)
        # R, t go to the camera unconverted, as in renderer.py:65-69
        self.cameras = PerspectiveCameras(in_ndc=False, device=self.device, R=R, T=t, K=K,
                                          image_size=torch.tensor([self.image_size]))
        self.raster_settings = RasterizationSettings(image_size=self.image_size, blur_radius=0.0, faces_per_pixel=1)
        self.lights = PointLights(device=self.device, location=[[0.0, 0.0, -3.0]])

    def load_meshes(self, files, textures=True):
        self.meshes = load_objs_as_meshes(files, device=self.device, load_textures=textures)

    def update_light_position(self, position):
        self.lights.location = torch.tensor([position], dtype=torch.float32)

    def build_color_renderer(self):
        self.color_renderer = MeshRenderer(
            rasterizer=MeshRasterizer(cameras=self.cameras, raster_settings=self.raster_settings),
            shader=SoftPhongShader(device=self.device, cameras=self.cameras, lights=self.lights))

    def render(self):
        return self.color_renderer(self.meshes)
