"""The libtorch RasterizeGaussians autograd Function (C++ render() surface) on the GPU:
its gradients equal the C-ABI backward, and render() with a GaussianModel trains."""
import numpy as np
import pytest
import torch

from conftest import pkg, rel_l2

pytestmark = pytest.mark.gpu


def _setup(P=4000, W=192, H=144, seed=3):
    gr, sc = pkg("graphics"), pkg("scene")
    cam = gr.synthetic_camera(W, H)
    return cam, sc.make_scene(cam, P, max_sh_degree=3, seed=seed), sc.make_dL_dpix(cam, seed=seed + 1)


def test_autograd_matches_cabi():
    cam, s, dpix = _setup()
    R = pkg("rasterizer")
    dev = "cuda"
    t = lambda a: torch.tensor(a, device=dev, requires_grad=True)
    means, opac, scales, rots, dc, rest = (t(s.means3D), t(s.opacities), t(s.scales), t(s.rotations),
                                           t(s.sh_dc), t(s.sh_rest))
    m2d = torch.zeros_like(means, requires_grad=True)
    color, radii = R.rasterize_gaussians(cam, means, m2d, opac, sh_dc=dc, sh_rest=rest, scales=scales,
                                         rotations=rots, sh_degree=3)
    (color * torch.tensor(dpix, device=dev)).sum().backward()
    cabi = R.CAbiRasterizer(dev)
    st = cabi.forward(cam, s.means3D, s.opacities, s.scales, s.rotations, s.sh_dc, s.sh_rest, sh_degree=3)
    assert torch.equal(st.color, color.detach())
    assert torch.equal(st.radii, radii)
    g = cabi.backward(st, dpix)
    pairs = dict(means3D=means, opacities=opac, scales=scales, rotations=rots, sh_dc=dc, sh_rest=rest,
                 means2D=m2d)
    for k, leaf in pairs.items():
        assert torch.equal(leaf.grad.reshape(g[k].shape), g[k]), k


def test_render_with_model_and_pipeline_flags():
    cam, s, dpix = _setup(P=3000)
    R, M = pkg("rasterizer"), pkg("model")
    model = M.GaussianModel.from_scene(s, "cuda")
    bg = torch.zeros(3, device="cuda")
    base = R.render(cam, model, R.PipelineParams(), bg)
    assert base["render"].shape == (3, cam.height, cam.width)
    assert torch.equal(base["visibility_filter"], base["radii"] > 0)
    # compute_cov3D_python and convert_SHs_python select the precomputed paths: same image
    alt = R.render(cam, model, R.PipelineParams(convert_SHs_python=True, compute_cov3D_python=True), bg)
    assert rel_l2(alt["render"].detach().cpu().numpy(), base["render"].detach().cpu().numpy()) < 1e-4
    # gradients reach every leaf through the activations, and a few Adam steps lower an L2 loss
    target = torch.rand_like(base["render"])
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    losses = []
    for _ in range(5):
        out = R.render(cam, model, R.PipelineParams(), bg)
        loss = ((out["render"] - target) ** 2).mean()
        opt.zero_grad()
        loss.backward()
        assert out["viewspace_points"].grad is not None
        losses.append(float(loss))
        opt.step()
    assert losses[-1] < losses[0]
    for p in model.parameters():
        assert p.grad is not None and bool(torch.isfinite(p.grad).all())


def test_precomputed_inputs_autograd():
    cam, s, dpix = _setup(P=1500)
    R, general = pkg("rasterizer"), pkg("general")
    dev = "cuda"
    means = torch.tensor(s.means3D, device=dev, requires_grad=True)
    cov = general.build_covariance_from_scaling_rotation(torch.tensor(s.scales, device=dev), 1.0,
                                                         torch.tensor(s.rotations, device=dev))
    cov = cov.detach().requires_grad_(True)
    cols = torch.rand((s.P, 3), device=dev, requires_grad=True)
    opac = torch.tensor(s.opacities, device=dev, requires_grad=True)
    m2d = torch.zeros_like(means, requires_grad=True)
    color, radii = R.rasterize_gaussians(cam, means, m2d, opac, colors_precomp=cols, cov3D_precomp=cov)
    (color * torch.tensor(dpix, device=dev)).sum().backward()
    for leaf in (means, cov, cols, opac, m2d):
        assert leaf.grad is not None and bool(torch.isfinite(leaf.grad).all())
    assert float(cov.grad.abs().sum()) > 0
