"""Diagnostic: capture -> restore -> continue, where do the trainers diverge?"""
import sys, os, tempfile
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import importlib
import torch
gr = importlib.import_module("3d_gaussian_splatting_amd.graphics")
sc = importlib.import_module("3d_gaussian_splatting_amd.scene")
T = importlib.import_module("3d_gaussian_splatting_amd.trainer")


def trainer(seed=0):
    cam = gr.synthetic_camera(160, 120)
    s = sc.make_scene(cam, 3000, max_sh_degree=3, seed=seed)
    tr = T.GaussianTrainer(s.means3D, s.sh_dc, s.sh_rest, s.raw_opacities, s.raw_scales, s.raw_rotations,
                           max_sh_degree=3, spatial_lr_scale=1.3)
    gt = torch.tensor(sc.make_dL_dpix(cam, seed=3), device="cuda") * 0.5 + 0.5
    return tr, cam, gt


a, cam, gt = trainer()
for it in range(1, 4):
    a.step(it, cam, gt, densify=False)
d = tempfile.mkdtemp()
path = os.path.join(d, "c.pth")
a.capture(path)
b, _, _ = trainer(seed=5)
b.restore(path)
md = lambda x, y: float((x - y).abs().max()) if x.shape == y.shape else "shape"
print("after restore", {k: md(a.params[k], b.params[k]) for k in a.params},
      {k: md(a.exp_avg[k], b.exp_avg[k]) for k in a.params}, a.steps, b.steps, a.lr, b.lr,
      a.active_sh_degree, b.active_sh_degree, a.spatial_lr_scale, b.spatial_lr_scale, flush=True)
print("stats", md(a.xyz_gradient_accum, b.xyz_gradient_accum), md(a.denom, b.denom), md(a.max_radii2D, b.max_radii2D))
for it in range(4, 6):
    oa = a.step(it, cam, gt, densify=False)
    ob = b.step(it, cam, gt, densify=False)
    print("iter", it, "img", md(oa["image"], ob["image"]), {k: md(a.params[k], b.params[k]) for k in a.params},
          a.lr["xyz"], b.lr["xyz"], flush=True)
