"""rel-L2 of the image and every gradient against the oracle on test_checkpoint_slots_deep_lists'
scene (64x64, P faint wide records, never terminating), for whichever libgsr_hip.so
GSR_HIP_LIB names: tells chunk-merging effects from f32 drift over deep lists.
usage: [GSR_HIP_LIB=...] python tests/diag_deep_lists.py P OPACITY  (a diagnostic, not collected)"""
import importlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
PKG = "3d_gaussian_splatting_amd"
pkg = lambda m: importlib.import_module(f"{PKG}.{m}")


def main():
    P, o = int(sys.argv[1]), float(sys.argv[2])
    gr, sc, R, native = pkg("graphics"), pkg("scene"), pkg("rasterizer"), pkg("native")
    import gsr_oracle as oracle
    oracle.build()
    cam = gr.synthetic_camera(64, 64)
    s = sc.make_scene(cam, P, max_sh_degree=1, seed=71)
    rng = np.random.default_rng(71)
    z = np.linspace(4.0, 8.0, P)
    xy = rng.uniform(-0.4, 0.4, (P, 2)) * z[:, None] * np.array([cam.tanfovx, cam.tanfovy])
    s.means3D = np.concatenate([xy, z[:, None]], 1).astype(np.float32)
    s.scales = np.full((P, 3), 6.0, np.float32)
    s.opacities = np.full((P, 1), o, np.float32)
    args = (cam, s.means3D, s.opacities, s.scales, s.rotations, s.sh_dc, s.sh_rest)
    rast = R.CAbiRasterizer("cuda")
    st = rast.forward(*args, sh_degree=1)
    f = oracle.forward(*args, sh_degree=1)
    dpix = sc.make_dL_dpix(cam, seed=72)
    g = rast.backward(st, dpix)
    gc = f.state.backward(dpix)
    rel = lambda a, b: float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))
    tiles = cam.grid[0] * cam.grid[1]
    term = st.view(native.VIEW_TERM, torch.int32, tiles * native.TERM_STRIDE).cpu().numpy().view(np.uint32)
    chunks = 1 + (term.reshape(tiles, -1)[:, 1:] != 0xFFFFFFFF).sum(1)
    out = {"lib": os.environ.get("GSR_HIP_LIB", "in-tree"), "P": P, "chunks_max": int(chunks.max()),
           "rgb": rel(st.color.cpu().numpy(), f.color)}
    for k in ("means2D", "opacities", "colors", "means3D", "sh_dc", "scales"):
        if k in g and k in gc:
            out[k] = rel(g[k].cpu().numpy().reshape(gc[k].shape), gc[k])
    print(out, flush=True)


if __name__ == "__main__":
    main()
