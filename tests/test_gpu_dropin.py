"""GPU: the C++ drop-in (lib/gsr_dropin, built from tests/cpp/dropin_main.cpp + gsr_torch.cpp with
-DGSR_NO_PYBIND) -- gsr::render<GaussianModel, PipelineParams>() compiled against the
reference's exact getter / PipelineParams / Camera surface -- runs one render -> L1 -> backward
-> Adam step, and every output equals the same step through the C ABI (CAbiRasterizer) with
torch autograd for the activations and torch.optim.Adam for the update.

Also checks gsr::RasterCamera::from_tensors against graphics.make_camera.  Cases: the default
pipeline; compute_cov3D_python with an integral modifier (the reference's
get_covariance(int) path); compute_cov3D_python with modifier 0.8 (must NOT be truncated to 0
by get_covariance(int): render() applies it in-kernel instead); convert_SHs_python."""
import os
import subprocess
import tempfile

import numpy as np
import pytest
import torch

from conftest import ROOT, pkg

pytestmark = pytest.mark.gpu
EXE = os.path.join(ROOT, "3d_gaussian_splatting_amd", "lib", "gsr_dropin")
LRS = {"xyz": 0.00016, "f_dc": 0.0025, "f_rest": 0.0025 / 20.0, "opacity": 0.05, "scaling": 0.005, "rotation": 0.001}


def _inputs(P=3000, W=160, H=120, D=3, seed=5):
    gr, sc = pkg("graphics"), pkg("scene")
    cam = gr.synthetic_camera(W, H)
    s = sc.make_scene(cam, P, max_sh_degree=3, seed=seed)
    target = (sc.make_dL_dpix(cam, seed=seed + 1) * 0.5 + 0.5).astype(np.float32)
    return cam, s, target


def _write_in(fin, cam, s, target, D, flags, smod):
    import math
    P, M = s.P, s.sh_rest.shape[1]
    fovx = 2 * math.atan(cam.tanfovx)
    fovy = 2 * math.atan(cam.tanfovy)
    with open(fin, "wb") as fh:
        fh.write(np.array([P, cam.width, cam.height, D, M, *flags], np.int32).tobytes())
        fh.write(np.concatenate([np.eye(3).ravel(), np.zeros(3), [fovx, fovy]]).astype(np.float64).tobytes())
        fh.write(np.array([smod], np.float32).tobytes())
        for a in (s.means3D, s.sh_dc, s.sh_rest, s.raw_opacities, s.raw_scales, s.raw_rotations, target):
            fh.write(np.ascontiguousarray(a, np.float32).tobytes())


def _exec(args):
    try:
        r = subprocess.run([EXE] + args, capture_output=True, text=True, timeout=150)
    except subprocess.TimeoutExpired as e:
        pytest.fail(f"gsr_dropin timed out; its progress:\n{e.stderr}")
    print(r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr


def _run_exe(cam, s, target, D, flags, smod):
    import math
    P, M = s.P, s.sh_rest.shape[1]
    fovx = 2 * math.atan(cam.tanfovx)
    fovy = 2 * math.atan(cam.tanfovy)
    with tempfile.TemporaryDirectory() as d:
        fin, fout = os.path.join(d, "in.bin"), os.path.join(d, "out.bin")
        with open(fin, "wb") as fh:
            fh.write(np.array([P, cam.width, cam.height, D, M, *flags], np.int32).tobytes())
            fh.write(np.concatenate([np.eye(3).ravel(), np.zeros(3), [fovx, fovy]]).astype(np.float64).tobytes())
            fh.write(np.array([smod], np.float32).tobytes())
            for a in (s.means3D, s.sh_dc, s.sh_rest, s.raw_opacities, s.raw_scales, s.raw_rotations, target):
                fh.write(np.ascontiguousarray(a, np.float32).tobytes())
        try:
            r = subprocess.run([EXE, fin, fout], capture_output=True, text=True, timeout=150)
        except subprocess.TimeoutExpired as e:
            pytest.fail(f"gsr_dropin timed out; its progress:\n{e.stderr}")
        print(r.stderr)
        assert r.returncode == 0, r.stdout + r.stderr
        raw = open(fout, "rb").read()
    H, W = cam.height, cam.width
    sizes = [("render", 3 * H * W, np.float32), ("radii", P, np.int32), ("means2D", 3 * P, np.float32),
             ("g_xyz", 3 * P, np.float32), ("g_f_dc", 3 * P, np.float32), ("g_f_rest", 3 * M * P, np.float32),
             ("g_opacity", P, np.float32), ("g_scaling", 3 * P, np.float32), ("g_rotation", 4 * P, np.float32),
             ("xyz", 3 * P, np.float32), ("f_dc", 3 * P, np.float32), ("f_rest", 3 * M * P, np.float32),
             ("opacity", P, np.float32), ("scaling", 3 * P, np.float32), ("rotation", 4 * P, np.float32),
             ("loss", 1, np.float32), ("camera", 37, np.float32)]
    out, off = {}, 0
    for name, n, dt in sizes:
        out[name] = np.frombuffer(raw, dt, n, off)
        off += n * np.dtype(dt).itemsize
    assert off == len(raw)
    return out


def _standin_covariance(q, s, mod):
    """The stand-in GaussianModel::get_covariance(int) of dropin_main.cpp, op for op (the
    reference's R S S^T R^T, general_utils.cpp:88-99), so both sides build bit-identical cov3D."""
    r, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R = torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y),
                     2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x),
                     2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], 1).view(-1, 3, 3)
    L = R * (mod * s).unsqueeze(1)
    S = torch.bmm(L, L.transpose(1, 2))
    return torch.stack([S[:, 0, 0], S[:, 0, 1], S[:, 0, 2], S[:, 1, 1], S[:, 1, 2], S[:, 2, 2]], 1)


def _camera_of(cam, c):
    """graphics.RasterCamera with the f32 fields gsr::RasterCamera::from_tensors produced."""
    gr = pkg("graphics")
    return gr.RasterCamera(width=cam.width, height=cam.height, tanfovx=float(c[0]), tanfovy=float(c[1]),
                           viewmatrix=np.array(c[2:18], np.float32), projmatrix=np.array(c[18:34], np.float32),
                           campos=np.array(c[34:37], np.float32))


def _reference_step(cam, s, target, D, flags, smod):
    """The same step through the C ABI + torch autograd + torch.optim.Adam (reference path)."""
    R, general = pkg("rasterizer"), pkg("general")
    dev = torch.device("cuda", 0)
    leaf = lambda a, shape: torch.tensor(np.asarray(a, np.float32).reshape(shape), device=dev, requires_grad=True)
    P, M = s.P, s.sh_rest.shape[1]
    p = {"xyz": leaf(s.means3D, (P, 3)), "f_dc": leaf(s.sh_dc, (P, 1, 3)), "f_rest": leaf(s.sh_rest, (P, M, 3)),
         "opacity": leaf(s.raw_opacities, (P, 1)), "scaling": leaf(s.raw_scales, (P, 3)),
         "rotation": leaf(s.raw_rotations, (P, 4))}
    sc = torch.exp(p["scaling"])
    q = torch.nn.functional.normalize(p["rotation"], dim=1)
    o = torch.sigmoid(p["opacity"])
    convert, cov_py = flags[0], flags[1]
    kw = dict(sh_degree=D)
    if cov_py and smod == round(smod):
        kw["cov3D_precomp"] = _standin_covariance(q, sc, int(smod))
    else:
        kw.update(scales=sc, rotations=q, scale_modifier=smod)
    if convert:
        dirs = p["xyz"] - torch.tensor(cam.campos, device=dev)
        dirs = dirs / dirs.norm(dim=1, keepdim=True)
        feats = torch.cat([p["f_dc"], p["f_rest"]], 1)
        kw["colors_precomp"] = torch.clamp_min(general.eval_sh(D, feats, dirs) + 0.5, 0.0)
        kw["sh_degree"] = 0
    else:
        kw.update(sh_dc=p["f_dc"], sh_rest=p["f_rest"])
    means2D = torch.zeros_like(p["xyz"], requires_grad=True)
    color, radii = R.rasterize_gaussians(cam, p["xyz"], means2D, o, **kw)
    gt = torch.tensor(target, device=dev)
    loss = torch.abs(color - gt).mean()
    loss.backward()
    grads = {k: v.grad.clone() for k, v in p.items()}
    opts = [torch.optim.Adam([p[k]], lr=LRS[k]) for k in p]
    for opt in opts:
        opt.step()
    return color.detach(), radii, means2D.grad, grads, {k: v.detach() for k, v in p.items()}, float(loss)


@pytest.mark.parametrize("flags,smod", [((0, 0, 0), 1.0), ((0, 1, 0), 1.0), ((0, 1, 0), 0.8), ((1, 0, 0), 1.0)],
                         ids=["default", "cov3D_python", "cov3D_python_mod0.8", "convert_SHs_python"])
def test_cpp_dropin_step_matches_cabi(flags, smod):
    assert os.path.exists(EXE), "run __graft_entry__.build()"
    cam, s, target = _inputs()
    D = 3
    out = _run_exe(cam, s, target, D, flags, smod)
    # RasterCamera::from_tensors on the Camera's float64 tensors (camera.cpp:66-71) agrees with
    # graphics.make_camera to f32 rounding; the reference step then uses its exact camera
    c = out["camera"]
    np.testing.assert_allclose(c[2:18], cam.viewmatrix, rtol=0, atol=1e-6)
    np.testing.assert_allclose(c[18:34], cam.projmatrix, rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(c[34:37], cam.campos, rtol=0, atol=1e-6)
    assert abs(c[0] - cam.tanfovx) <= 1e-6 and abs(c[1] - cam.tanfovy) <= 1e-6
    cam = _camera_of(cam, c)
    color, radii, m2d, grads, params, loss = _reference_step(cam, s, target, D, flags, smod)
    n = lambda t: t.detach().cpu().numpy().ravel()
    np.testing.assert_allclose(out["render"], n(color), rtol=0, atol=1e-6)
    np.testing.assert_array_equal(out["radii"], n(radii))
    assert abs(out["loss"][0] - loss) <= 1e-6 * max(abs(loss), 1.0)
    rel = lambda a, b: float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))
    assert rel(out["means2D"], n(m2d)) <= 1e-5
    for k in grads:
        assert rel(out["g_" + k], n(grads[k])) <= 1e-5, k
        # Adam's first step moves each entry by ~lr g / (|g| + eps): entries with |g| near eps
        # turn the gradients' 1e-5-level agreement into update differences of the same order
        assert rel(out[k], n(params[k])) <= 1e-5, k
    if flags[1] and smod != round(smod):
        # a truncated modifier (get_covariance(int(0.8)) = zero covariances) would have culled
        # every Gaussian: the render must show them
        assert int((out["radii"] > 0).sum()) > 0.5 * s.P


LOOP_ITERS = 4


def test_cpp_dropin_loop_sync_free_fused():
    """The drop-in pieces of csrc/torch/gsr_trainer.h in the reference's autograd loop: LOOP_ITERS
    iterations of gsr::render under a gsr::BinningCapacity -- only the first render reads K back
    (num_rendered -1 afterwards: the bound is on the device), gsr::read_num_rendered of the last
    render equals the exact K -- then gsr::photometric_loss (L1 + D-SSIM autograd Function),
    backward, gsr::densify_stats and gsr::fused_adam_step on the six torch::optim::Adam (one
    launch on libtorch's own Adam state).  Against the same loop through the C ABI with torch
    autograd, the upstream torch SSIM formulation (oracle/train_oracle.py) and torch.optim.Adam:
    losses within 1e-5 relative, parameters and statistics within 1e-4 relative L2 after the
    last step (each Adam step turns gradient differences near eps into update differences)."""
    import train_oracle  # test infrastructure: the upstream loss formulation
    assert os.path.exists(EXE), "run __graft_entry__.build()"
    R = pkg("rasterizer")
    cam, s, target = _inputs(P=4000, W=192, H=128)
    D, P, M = 3, s.P, s.sh_rest.shape[1]
    with tempfile.TemporaryDirectory() as d:
        fin, fout = os.path.join(d, "in.bin"), os.path.join(d, "out.bin")
        _write_in(fin, cam, s, target, D, (0, 0, 0), 1.0)
        _exec([fin, fout, str(LOOP_ITERS)])
        raw = open(fout, "rb").read()
    H, W = cam.height, cam.width
    ints = np.frombuffer(raw, np.int32, 2 * LOOP_ITERS + 3)
    host_k, caps = ints[0:2 * LOOP_ITERS:2], ints[1:2 * LOOP_ITERS:2]
    k_last, overflows, exact_reads = ints[2 * LOOP_ITERS:]
    off = ints.nbytes
    sizes = [("stats", 3 * LOOP_ITERS), ("render", 3 * H * W), ("xyz", 3 * P), ("f_dc", 3 * P), ("f_rest", 3 * M * P),
             ("opacity", P), ("scaling", 3 * P), ("rotation", 4 * P), ("max_radii2D", P), ("accum", P), ("denom", P)]
    out = {}
    for name, n in sizes:
        out[name] = np.frombuffer(raw, np.float32, n, off)
        off += 4 * n
    assert off == len(raw)
    # sync-free: one exact read (the first render), then bounded renders whose K stays on the device
    assert host_k[0] > 0 and all(k == -1 for k in host_k[1:]), host_k
    assert all(c > host_k[0] for c in caps[1:]) and overflows == 0 and exact_reads == 1

    # the same loop through the C ABI + torch autograd + upstream torch SSIM + torch.optim.Adam
    dev = torch.device("cuda", 0)
    leaf = lambda a, shape: torch.tensor(np.asarray(a, np.float32).reshape(shape), device=dev, requires_grad=True)
    p = {"xyz": leaf(s.means3D, (P, 3)), "f_dc": leaf(s.sh_dc, (P, 1, 3)), "f_rest": leaf(s.sh_rest, (P, M, 3)),
         "opacity": leaf(s.raw_opacities, (P, 1)), "scaling": leaf(s.raw_scales, (P, 3)),
         "rotation": leaf(s.raw_rotations, (P, 4))}
    opts = [torch.optim.Adam([p[k]], lr=LRS[k]) for k in p]
    max_r = torch.zeros(P, device=dev)
    accum = torch.zeros(P, device=dev)
    denom = torch.zeros(P, device=dev)
    gt = torch.tensor(target, device=dev)
    rast = R.CAbiRasterizer(dev)
    for it in range(LOOP_ITERS):
        m2d = torch.zeros_like(p["xyz"], requires_grad=True)
        color, radii = R.rasterize_gaussians(cam, p["xyz"], m2d, torch.sigmoid(p["opacity"]), sh_dc=p["f_dc"],
                                             sh_rest=p["f_rest"], scales=torch.exp(p["scaling"]),
                                             rotations=torch.nn.functional.normalize(p["rotation"], dim=1),
                                             sh_degree=D)
        if it == LOOP_ITERS - 1:  # K of the last render (the one gsr::read_num_rendered read)
            k_ref = rast.forward(cam, p["xyz"].detach(), torch.sigmoid(p["opacity"]).detach(),
                                 scales=torch.exp(p["scaling"]).detach(),
                                 rotations=torch.nn.functional.normalize(p["rotation"], dim=1).detach(),
                                 sh_dc=p["f_dc"].detach(), sh_rest=p["f_rest"].detach(), sh_degree=D).num_rendered
        loss, l1, ssim, dimg = train_oracle.ssim_loss(color.detach().cpu().numpy(), target, 0.2)
        st = out["stats"][3 * it:3 * it + 3]
        assert abs(st[0] - loss) <= 1e-5 * abs(loss) and abs(st[1] - l1) <= 1e-5 * abs(l1), (it, st, loss, l1)
        color.backward(torch.tensor(dimg, device=dev))
        with torch.no_grad():
            vis = radii > 0
            max_r[vis] = torch.maximum(max_r[vis], radii[vis].float())
            accum[vis] += m2d.grad[vis, :2].norm(dim=-1)
            denom[vis] += 1
        for o in opts:
            o.step()
            o.zero_grad()
    # the parameters agree to ~1e-5, so the instance counts may differ by a few rect edges
    assert abs(int(k_last) - k_ref) <= 1e-3 * k_ref, (k_last, k_ref)
    rel = lambda a, b: float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))
    n = lambda t: t.detach().cpu().numpy().ravel()
    for k in p:
        assert rel(out[k], n(p[k])) <= 1e-4, (k, rel(out[k], n(p[k])))
    np.testing.assert_array_equal(out["max_radii2D"], n(max_r))
    np.testing.assert_array_equal(out["denom"], n(denom))
    assert rel(out["accum"], n(accum)) <= 1e-4
