"""mi355r — MI355X-native differentiable mesh rasterizer (drop-in for the
render()/backward path of YufengJin/torch_renderer)."""
from .structures import Meshes, TexturesUV, TexturesVertex  # noqa: F401
from .io import load_obj, load_objs_as_meshes  # noqa: F401
from .cameras import PerspectiveCameras, FoVPerspectiveCameras  # noqa: F401
from .transforms import (quaternion_to_matrix, matrix_to_quaternion, look_at_view_transform,  # noqa: F401
                         look_at_rotation)

__version__ = "0.1.0"
from .mesh_renderer import (RasterizationSettings, MeshRasterizer, MeshRenderer, Fragments, rasterize,  # noqa: F401
                            PointLights, AmbientLights, Materials, BlendParams, SoftPhongShader,
                            SoftSilhouetteShader, HardPhongShader)
