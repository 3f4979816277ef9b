#!/usr/bin/env python3
"""Check that chunked B1 (multi-GPU bands) matches unchunked B1 on a 1080p band with long
tile lists: prints the relative L2 difference of grad2d and the forward image."""
import importlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "3d_gaussian_splatting_amd"
gr = importlib.import_module(f"{PKG}.graphics")
sc = importlib.import_module(f"{PKG}.scene")
R = importlib.import_module(f"{PKG}.rasterizer")


def run(chunk, P=1_000_000, band=(25, 34)):
    os.environ["GSR_CHUNK"] = str(chunk)
    dev = torch.device("cuda", 0)
    cam = gr.synthetic_camera(1920, 1080)
    scene = sc.make_scene(cam, P, max_sh_degree=3, seed=0)
    t = lambda a: torch.tensor(a, device=dev)
    rast = R.CAbiRasterizer(dev)
    st = rast.forward(cam, means3D=t(scene.means3D), opacities=t(scene.opacities), scales=t(scene.scales),
                      rotations=t(scene.rotations), sh_dc=t(scene.sh_dc), sh_rest=t(scene.sh_rest), sh_degree=3,
                      tile_rows=band)
    g2 = rast.backward_blend(st, t(sc.make_dL_dpix(cam, seed=1)))
    torch.cuda.synchronize()
    return st.color.clone(), g2.clone()


c0, g0 = run(0)
c1, g1 = run(1)
rel = float((g1 - g0).norm() / g0.norm())
print(f"image equal: {torch.equal(c0, c1)}  grad2d rel L2 chunked vs unchunked: {rel:.3e}")
sys.exit(0 if torch.equal(c0, c1) and rel < 1e-5 else 1)
