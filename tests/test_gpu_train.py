"""GPU parity of the training-step kernels (include/gsr/gsr_train.h)
against the CPU restatements in oracle/train_oracle.py, through the C ABI.

Tolerances (floating point, stated here):
  * loss value / L1 / SSIM: relative 1e-5 (f32 sums in a different order);
  * dL/dimg: relative L2 1e-5, element-wise 1e-5 of max |dL/dimg|;
  * activations: element-wise relative 1e-6;
  * Adam (params after 3 steps, activation backward fused): relative 1e-5 of max(|p|, 1e-3);
  * densify statistics: relative 1e-6; compaction / row gathers / prune: bit-exact;
  * densify_and_prune: bit-exact rows except the split children's positions (torch bmm on
    the device vs the CPU), relative 1e-5;
  * one full training step (render + loss + backward + Adam) vs the CPU composite
    (oracle rasterizer + torch loss + libtorch-Adam restatement): relative 1e-4 on the updated
    leaves' change.
"""
import numpy as np
import pytest
import torch

from conftest import pkg, rel_l2

import train_oracle as T

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def K():
    return pkg("trainer").TrainKernels(DEV)


def _t(a):
    return torch.as_tensor(np.ascontiguousarray(a, dtype=np.float32), device=DEV)


@pytest.mark.parametrize("shape", [(3, 16, 16), (3, 70, 101), (1, 33, 200), (3, 1080, 1920)])
def test_loss_matches_torch(K, shape):
    rng = np.random.default_rng(sum(shape))
    gt = rng.random(shape, dtype=np.float32)
    img = np.clip(gt + 0.1 * rng.standard_normal(shape).astype(np.float32), 0, 1)
    loss, l1, s, g = T.ssim_loss(img, gt, 0.2)
    stats, maps = K.loss_forward(_t(img), _t(gt), 0.2)
    dimg = K.loss_backward(_t(img), _t(gt), 0.2, maps).cpu().numpy()
    st = stats.cpu().numpy().astype(np.float64)
    for a, b in zip(st, (loss, l1, s)):
        assert abs(a - b) <= 1e-5 * abs(b), (st, loss, l1, s)
    assert rel_l2(dimg, g) <= 1e-5
    assert np.max(np.abs(dimg - g)) <= 1e-5 * np.max(np.abs(g)) + 1e-12


def test_loss_is_deterministic(K):
    rng = np.random.default_rng(7)
    img, gt = _t(rng.random((3, 200, 300))), _t(rng.random((3, 200, 300)))
    a, m = K.loss_forward(img, gt, 0.2)
    b, m2 = K.loss_forward(img, gt, 0.2)
    assert torch.equal(a, b)
    assert torch.equal(K.loss_backward(img, gt, 0.2, m), K.loss_backward(img, gt, 0.2, m2))


def test_activate_matches_torch(K):
    rng = np.random.default_rng(8)
    P = 5003
    s, q, o = rng.standard_normal((P, 3)), rng.standard_normal((P, 4)), rng.standard_normal((P, 1)) * 3
    a = K.activate(_t(s), _t(q), _t(o))
    ref = T.activate(s, q, o)
    for x, y in zip(a, ref):
        x = x.cpu().numpy()
        assert np.max(np.abs(x - y) / np.maximum(np.abs(y), 1e-30)) <= 1e-6


def test_adam_matches_libtorch_restatement(K):
    """Three steps of the six groups in one launch each, activation backward fused, against
    autograd activation backward + the libtorch Adam restatement (itself pinned to
    torch.optim.Adam in test_train_oracle.py)."""
    rng = np.random.default_rng(9)
    P = 4099
    shapes = {"xyz": (P, 3), "f_dc": (P, 1, 3), "f_rest": (P, 15, 3), "opacity": (P, 1), "scaling": (P, 3),
              "rotation": (P, 4)}
    acts = pkg("trainer").ACTS
    lrs = {"xyz": 1.6e-4, "f_dc": 2.5e-3, "f_rest": 1.25e-4, "opacity": 0.05, "scaling": 5e-3, "rotation": 1e-3}
    p_cpu = {k: rng.standard_normal(s).astype(np.float32) for k, s in shapes.items()}
    m_cpu = {k: np.zeros(s, np.float32) for k, s in shapes.items()}
    v_cpu = {k: np.zeros(s, np.float32) for k, s in shapes.items()}
    p_gpu = {k: _t(v) for k, v in p_cpu.items()}
    m_gpu = {k: torch.zeros_like(v) for k, v in p_gpu.items()}
    v_gpu = {k: torch.zeros_like(v) for k, v in p_gpu.items()}
    for step in (1, 2, 3):
        g_act = {k: (rng.standard_normal(s) * 10.0 ** rng.uniform(-5, -1, s)).astype(np.float32)
                 for k, s in shapes.items()}
        ds, dq, do = T.raw_grads(p_cpu["scaling"], p_cpu["rotation"], p_cpu["opacity"], g_act["scaling"],
                                 g_act["rotation"], g_act["opacity"])
        g_raw = dict(g_act, scaling=ds, rotation=dq, opacity=do)
        for k in shapes:
            T.adam_step(p_cpu[k], g_raw[k], m_cpu[k], v_cpu[k], step, lrs[k])
        K.adam_step([dict(param=p_gpu[k], grad=_t(g_act[k]), exp_avg=m_gpu[k], exp_avg_sq=v_gpu[k],
                          act=acts[k], step=step, lr=lrs[k]) for k in shapes])
    for k in shapes:
        a = p_gpu[k].cpu().numpy()
        err = np.max(np.abs(a - p_cpu[k]) / np.maximum(np.abs(p_cpu[k]), 1e-3))
        assert err <= 1e-5, (k, err)
        assert rel_l2(m_gpu[k].cpu().numpy(), m_cpu[k]) <= 1e-5, k


def test_densify_stats(K):
    rng = np.random.default_rng(10)
    P = 10007
    radii = rng.integers(-1, 30, P).astype(np.int32)
    radii[radii < 0] = 0
    dm = rng.standard_normal((P, 3)).astype(np.float32) * 1e-3
    maxr, acc, den = rng.random(P).astype(np.float32) * 20, rng.random(P).astype(np.float32), np.ones(P, np.float32)
    tm, ta, td = _t(maxr), _t(acc), _t(den)
    K.densify_stats(torch.as_tensor(radii, device=DEV), _t(dm), tm, ta, td)
    vis = radii > 0
    maxr[vis] = np.maximum(maxr[vis], radii[vis].astype(np.float32))
    acc[vis] += np.sqrt(dm[vis, 0] ** 2 + dm[vis, 1] ** 2)
    den[vis] += 1
    np.testing.assert_array_equal(tm.cpu().numpy(), maxr)
    np.testing.assert_allclose(ta.cpu().numpy(), acc, rtol=1e-6)
    np.testing.assert_array_equal(td.cpu().numpy(), den)


def test_step_guard_skips_truncated_iterations(K):
    """gsr_adam_step_guarded / gsr_densify_stats_guarded: with the render's K above the bound it
    ran under, nothing changes (the truncated iteration is dropped on the device); at or below
    it, the guarded calls equal the unguarded ones bit for bit."""
    rng = np.random.default_rng(11)
    P = 5003
    p0 = rng.standard_normal((P, 3)).astype(np.float32)
    g = (rng.standard_normal((P, 3)) * 1e-2).astype(np.float32)
    radii = rng.integers(0, 30, P).astype(np.int32)
    dm = (rng.standard_normal((P, 3)) * 1e-3).astype(np.float32)
    acts = pkg("trainer").ACTS
    outs = {}
    for label, k in (("over", 1001), ("at", 1000), ("none", None)):
        p, m, v = _t(p0), torch.zeros(P, 3, device=DEV), torch.zeros(P, 3, device=DEV)
        stats = [torch.zeros(P, device=DEV) for _ in range(3)]
        guard = None if k is None else (torch.tensor([k], dtype=torch.int32, device=DEV), 1000)
        K.adam_step([dict(param=p, grad=_t(g), exp_avg=m, exp_avg_sq=v, act=acts["xyz"], step=1, lr=1e-3)],
                    guard=guard)
        K.densify_stats(torch.as_tensor(radii, device=DEV), _t(dm), *stats, guard=guard)
        outs[label] = [p, m, v] + stats
    for t, t0 in zip(outs["over"], [_t(p0)] + [torch.zeros_like(outs["over"][1])] * 2 +
                     [torch.zeros(P, device=DEV)] * 3):
        assert torch.equal(t, t0)
    for a, b in zip(outs["at"], outs["none"]):
        assert torch.equal(a, b)
    assert not torch.equal(outs["at"][0], _t(p0))


@pytest.mark.parametrize("n,frac", [(1, 1.0), (1023, 0.5), (1024, 0.0), (4097, 1.0), (1_000_003, 0.3)])
def test_compact_and_gather_bit_exact(K, n, frac):
    g = torch.Generator().manual_seed(n)
    mask = torch.rand(n, generator=g) < frac
    idx = K.compact_index(mask.to(DEV))
    ref = torch.nonzero(mask).flatten().to(torch.int32)
    assert torch.equal(idx.cpu(), ref)
    a, b = torch.randn(n, 15, 3, generator=g), torch.randn(n, generator=g)
    out = K.gather_rows([a.to(DEV), b.to(DEV)], idx)
    assert torch.equal(out[0].cpu(), a[mask]) and torch.equal(out[1].cpu(), b[mask])


def _trainer_from_state(st, extent=1.0):
    Tr = pkg("trainer")
    tr = Tr.GaussianTrainer(st["xyz"], st["f_dc"], st["f_rest"], st["opacity"], st["scaling"], st["rotation"],
                            max_sh_degree=3, device=DEV)
    for k in Tr.GROUPS:
        tr.exp_avg[k] = st["m_" + k].to(DEV).contiguous()
        tr.exp_avg_sq[k] = st["v_" + k].to(DEV).contiguous()
    tr.xyz_gradient_accum = st["grad_accum"].to(DEV)
    tr.denom = st["denom"].to(DEV)
    tr.max_radii2D = st["max_radii2D"].to(DEV)
    tr.cameras_extent = extent
    return tr


def _state(n, seed=11):
    g = torch.Generator().manual_seed(seed)
    st = {"xyz": torch.randn(n, 3, generator=g), "f_dc": torch.randn(n, 1, 3, generator=g),
          "f_rest": torch.randn(n, 15, 3, generator=g), "opacity": torch.randn(n, 1, generator=g) * 3,
          "scaling": torch.log(torch.rand(n, 3, generator=g) * 0.05 + 1e-3),
          "rotation": torch.randn(n, 4, generator=g)}
    for k in list(st):
        st["m_" + k] = torch.randn_like(st[k])
        st["v_" + k] = torch.rand_like(st[k])
    st["denom"] = torch.randint(0, 3, (n,), generator=g).float()
    st["grad_accum"] = torch.rand(n, generator=g) * 4e-4 * st["denom"]
    st["max_radii2D"] = torch.randint(0, 40, (n,), generator=g).float()
    return st


@pytest.mark.parametrize("max_screen", [None, 20])
def test_densify_and_prune_matches_oracle(max_screen):
    st = _state(3000)
    thr, ext, pd = 2e-4, 1.0, 0.01
    n_split = T.split_count(st, thr, ext, pd)
    samples = torch.randn(2 * n_split, 3, generator=torch.Generator().manual_seed(5))
    ref = T.densify_and_prune(st, thr, 0.005, ext, max_screen, pd, samples)
    tr = _trainer_from_state(st, ext)
    tr.densify_and_prune(thr, 0.005, ext, max_screen, split_samples=samples.to(DEV))
    Tr = pkg("trainer")
    for k in Tr.GROUPS:
        a = tr.params[k].cpu()
        assert a.shape == ref[k].shape, (k, a.shape, ref[k].shape)
        if k == "xyz" or k == "scaling":
            assert rel_l2(a.numpy(), ref[k].numpy()) <= 1e-5, k
        else:
            assert torch.equal(a, ref[k]), k
        assert torch.equal(tr.exp_avg[k].cpu(), ref["m_" + k]), k
        assert torch.equal(tr.exp_avg_sq[k].cpu(), ref["v_" + k]), k
    for a, b in ((tr.xyz_gradient_accum, "grad_accum"), (tr.denom, "denom"), (tr.max_radii2D, "max_radii2D")):
        assert torch.equal(a.cpu(), ref[b])


def test_training_step_matches_cpu_composite(oracle):
    """One iteration on the GPU (activate -> gsr_forward -> loss -> gsr_backward -> stats ->
    fused Adam) against the CPU composite at a small size."""
    gr, sc, Tr = pkg("graphics"), pkg("scene"), pkg("trainer")
    cam = gr.synthetic_camera(160, 120)
    s = sc.make_scene(cam, 3000, max_sh_degree=3, seed=3)
    rng = np.random.default_rng(4)
    gt = rng.random((3, 120, 160)).astype(np.float32)
    tr = Tr.GaussianTrainer(s.means3D, s.sh_dc, s.sh_rest, s.raw_opacities.reshape(-1, 1), s.raw_scales,
                            s.raw_rotations, max_sh_degree=3, device=DEV)
    tr.active_sh_degree = 3
    before = {k: v.cpu().numpy().copy() for k, v in tr.params.items()}
    out = tr.step(1, cam, _t(gt), densify=False)
    # CPU composite
    sc_, q_, o_ = T.activate(s.raw_scales, s.raw_rotations, s.raw_opacities.reshape(-1, 1))
    f = oracle.forward(cam, s.means3D, o_.reshape(-1), sc_, q_, s.sh_dc, s.sh_rest, sh_degree=3)
    loss, l1, ssim_v, dimg = T.ssim_loss(f.color.astype(np.float32), gt, 0.2)
    st = out["stats"].cpu().numpy()
    assert abs(st[0] - loss) <= 1e-4 * abs(loss)
    g = f.state.backward(dimg.astype(np.float64))
    ds, dq, do = T.raw_grads(s.raw_scales, s.raw_rotations, s.raw_opacities.reshape(-1, 1), g["scales"],
                             g["rotations"], g["opacities"].reshape(-1, 1))
    graw = {"xyz": g["means3D"], "f_dc": g["sh_dc"], "f_rest": g["sh_rest"], "opacity": do, "scaling": ds,
            "rotation": dq}
    lr = dict(tr.lr)
    for k in Tr.GROUPS:
        p = before[k].copy()
        m, v = np.zeros_like(p), np.zeros_like(p)
        T.adam_step(p, graw[k].reshape(p.shape).astype(np.float32), m, v, 1, lr[k])
        # Adam's first step moves every element by ~lr sign(g): compare the moves on elements
        # whose gradient is not at round-off level
        d_gpu = tr.params[k].cpu().numpy() - before[k]
        d_cpu = p - before[k]
        big = np.abs(graw[k].reshape(p.shape)) > 1e-3 * np.max(np.abs(graw[k])) + 1e-20
        assert rel_l2(d_gpu[big], d_cpu[big]) <= 1e-4, k
