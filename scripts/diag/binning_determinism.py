"""Diagnostic: does a trainer step depend on the binning bound (exact vs bounded sizing)?"""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import importlib
import torch
gr = importlib.import_module("3d_gaussian_splatting_amd.graphics")
sc = importlib.import_module("3d_gaussian_splatting_amd.scene")
T = importlib.import_module("3d_gaussian_splatting_amd.trainer")
R = importlib.import_module("3d_gaussian_splatting_amd.rasterizer")

cam = gr.synthetic_camera(160, 120)
s = sc.make_scene(cam, 3000, max_sh_degree=3, seed=0)
gt = torch.tensor(sc.make_dL_dpix(cam, seed=3), device="cuda") * 0.5 + 0.5
mk = lambda: T.GaussianTrainer(s.means3D, s.sh_dc, s.sh_rest, s.raw_opacities, s.raw_scales, s.raw_rotations,
                               max_sh_degree=3, spatial_lr_scale=1.3)
a, b = mk(), mk()
for it in range(1, 6):
    a.step(it, cam, gt, densify=False)
    b.binning.reset()
    b.step(it, cam, gt, densify=False)
    diff = {k: float((a.params[k] - b.params[k]).abs().max()) for k in a.params}
    print("iter", it, "cap_a", a.binning.cap, diff, flush=True)
# raw render: exact vs bounded, same inputs
rast = R.CAbiRasterizer("cuda")
args = (cam, s.means3D, s.opacities, s.scales, s.rotations, s.sh_dc, s.sh_rest)
dp = sc.make_dL_dpix(cam, seed=1)
e = rast.forward(*args, sh_degree=3)
K = e.num_rendered
ge = rast.backward(e, dp)
for cap in (K, K + 1, 2 * K, 8 * K, 20 * K):
    st = rast.forward(*args, sh_degree=3, max_rendered=cap)
    g = rast.backward(st, dp)
    print("cap", cap, "K", K, "color eq", torch.equal(st.color, e.color),
          {k: torch.equal(g[k], ge[k]) for k in ge}, flush=True)
