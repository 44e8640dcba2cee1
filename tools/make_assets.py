"""Convert the reference's mesh assets (data/*.obj, data/cow_mesh/*) into compact
.npz files under assets/ (they must travel to the GPU box, where /root/reference
does not exist). Parsed with torch_renderer_amd.io.load_obj; the texture is kept
as uint8 so the float map (uint8 / 255) is reproduced exactly.

    python tools/make_assets.py [/root/reference/data]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from torch_renderer_amd.io import load_obj  # noqa: E402

SRC = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/data"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "assets")
MESHES = {"sphere": "sphere.obj", "teapot": "teapot.obj", "dolphin": "dolphin.obj", "cow": "cow_mesh/cow.obj"}

os.makedirs(OUT, exist_ok=True)
for name, rel in MESHES.items():
    verts, faces, aux = load_obj(os.path.join(SRC, rel), load_textures=True)
    d = {"verts": verts.numpy().astype(np.float32), "faces": faces.verts_idx.numpy().astype(np.int32)}
    if aux.verts_uvs is not None:
        d["verts_uvs"] = aux.verts_uvs.numpy().astype(np.float32)
        d["faces_uvs"] = faces.textures_idx.numpy().astype(np.int32)
    if aux.texture_images:
        img = next(iter(aux.texture_images.values())).numpy()
        d["texture_u8"] = np.round(img * 255.0).astype(np.uint8)
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **d)
    print(name, {k: v.shape for k, v in d.items()})
