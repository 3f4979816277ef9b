"""CPU checks of the training-step oracle (oracle/train_oracle.py) and the host logic of the
trainer: loss closed forms and finite differences, libtorch-Adam
restatement against torch.optim.Adam, the reference's LR-schedule KATs, densification
bookkeeping.  No GPU."""
import math

import numpy as np
import pytest
import torch

from conftest import pkg

import train_oracle as T


def test_ssim_identical_images_is_one():
    rng = np.random.default_rng(0)
    img = rng.random((3, 20, 23), dtype=np.float32)
    loss, l1, s, g = T.ssim_loss(img, img.copy(), 0.2)
    assert l1 == 0.0
    assert abs(s - 1.0) < 1e-6
    assert abs(loss) < 1e-6


def test_ssim_constant_images_closed_form():
    # x = a, y = b everywhere, away from the border: S = (2ab + C1) / (a^2 + b^2 + C1) (the
    # sigma terms vanish); zero padding lowers the border, so compare the interior via a
    # large image whose border share is small
    a, b = 0.7, 0.4
    x = np.full((1, 200, 200), a, np.float32)
    y = np.full((1, 200, 200), b, np.float32)
    _, l1, s, _ = T.ssim_loss(x, y, 0.2)
    assert abs(l1 - 0.3) < 1e-6
    C1 = 0.01 ** 2
    inner = (2 * a * b + C1) / (a * a + b * b + C1)
    assert abs(s - inner) < 0.02  # border rows/cols (5 of 200 per side) shift the mean slightly


def test_loss_gradient_matches_finite_differences():
    rng = np.random.default_rng(1)
    x = rng.random((3, 13, 17))
    y = rng.random((3, 13, 17))
    _, _, _, g = T.ssim_loss(x, y, 0.2, dtype=torch.float64)
    h = 1e-6
    for (c, i, j) in [(0, 0, 0), (1, 6, 8), (2, 12, 16), (0, 3, 11)]:
        xp, xm = x.copy(), x.copy()
        xp[c, i, j] += h
        xm[c, i, j] -= h
        lp = T.ssim_loss(xp, y, 0.2, dtype=torch.float64)[0]
        lm = T.ssim_loss(xm, y, 0.2, dtype=torch.float64)[0]
        fd = (lp - lm) / (2 * h)
        assert abs(fd - g[c, i, j]) <= 1e-6 * max(1.0, abs(fd)) + 1e-9, (c, i, j, fd, g[c, i, j])


@pytest.mark.parametrize("steps", [1, 5])
def test_adam_restatement_matches_torch(steps):
    rng = np.random.default_rng(2)
    p0 = rng.standard_normal(1000).astype(np.float32)
    p = torch.tensor(p0.copy(), requires_grad=True)
    opt = torch.optim.Adam([p], lr=1e-3, foreach=False)
    pn, m, v = p0.copy(), np.zeros_like(p0), np.zeros_like(p0)
    for s in range(1, steps + 1):
        g = (rng.standard_normal(1000) * 10.0 ** rng.uniform(-6, 0, 1000)).astype(np.float32)
        p.grad = torch.tensor(g)
        opt.step()
        T.adam_step(pn, g, m, v, s, 1e-3)
    ref = p.detach().numpy()
    assert np.max(np.abs(pn - ref) / np.maximum(np.abs(ref), 1e-3)) < 1e-5


def test_normalize_grad_is_tangent():
    rng = np.random.default_rng(3)
    q = rng.standard_normal((50, 4)).astype(np.float32)
    d = rng.standard_normal((50, 4)).astype(np.float32)
    _, gq, _ = T.raw_grads(np.zeros((50, 3)), q, np.zeros((50, 1)), np.zeros((50, 3)), d, np.zeros((50, 1)))
    # d/dq of q/|q| is orthogonal to q
    assert np.max(np.abs(np.sum(gq * q, axis=1))) < 1e-5


def test_expon_lr_func_reference_kats():
    """src/utils/general_utils.cpp:306-332 (the reference's own BOOST checks)."""
    f = pkg("general").get_expon_lr_func
    assert f(0.0, 0.0, 100, 0.5, 1000)(1) == 0.0
    assert math.isclose(f(0.1, 0.01, 100, 0.5, 1000)(0), 0.05, rel_tol=1e-7)
    assert math.isclose(f(0.1, 0.01, 0, 0.5, 1000)(0), 0.1, rel_tol=1e-7)
    # log-linear decay to lr_final at max_steps
    assert math.isclose(f(0.1, 0.01, 0, 1.0, 1000)(1000), 0.01, rel_tol=1e-9)
    assert math.isclose(f(0.1, 0.01, 0, 1.0, 1000)(500), math.sqrt(0.1 * 0.01), rel_tol=1e-9)


def test_optimization_params_defaults_match_reference():
    """src/arguments/params.h:50-68: the same fields and defaults; the float fields hold the
    values of the reference's C++ floats (what gsr::OptimizationParams, the reference's own
    struct, holds in the C++ loop)."""
    O = pkg("trainer").OptimizationParams()
    f = lambda x: float(np.float32(x))
    assert (O.iterations, O.position_lr_max_steps, O.densification_interval, O.opacity_reset_interval,
            O.densify_from_iter, O.densify_until_iter) == (30000, 30000, 100, 3000, 500, 15000)
    assert O.lambda_dssim == f(0.2) and O.percent_dense == f(0.01) and O.densify_grad_threshold == f(0.0002)
    assert (O.position_lr_init, O.position_lr_final, O.position_lr_delay_mult) == (f(0.00016), f(0.0000016), f(0.01))
    assert (O.feature_lr, O.opacity_lr, O.scaling_lr, O.rotation_lr) == (f(0.0025), f(0.05), f(0.005), f(0.001))


def _state(n, seed=4):
    g = torch.Generator().manual_seed(seed)
    st = {"xyz": torch.randn(n, 3, generator=g), "f_dc": torch.randn(n, 1, 3, generator=g),
          "f_rest": torch.randn(n, 15, 3, generator=g), "opacity": torch.randn(n, 1, generator=g) * 3,
          "scaling": torch.log(torch.rand(n, 3, generator=g) * 0.05 + 1e-3),
          "rotation": torch.randn(n, 4, generator=g)}
    for k in list(st):
        st["m_" + k] = torch.randn_like(st[k])
        st["v_" + k] = torch.rand_like(st[k])
    st["grad_accum"] = torch.rand(n, generator=g) * 4e-4
    st["denom"] = torch.randint(0, 3, (n,), generator=g).float()
    st["max_radii2D"] = torch.randint(0, 40, (n,), generator=g).float()
    return st


def test_densify_oracle_bookkeeping():
    st = _state(500)
    thr, ext, pd = 2e-4, 1.0, 0.01
    grads = st["grad_accum"] / st["denom"]
    grads[grads.isnan()] = 0.0
    big = torch.exp(st["scaling"]).max(1).values > pd * ext
    n_clone = int(((grads >= thr) & ~big).sum())
    n_split = T.split_count(st, thr, ext, pd)
    assert n_split == int(((grads >= thr) & big).sum())
    samples = torch.randn(2 * n_split, 3)
    out = T.densify_and_prune(st, thr, 0.005, ext, None, pd, samples)
    n_low = int((torch.sigmoid(st["opacity"]) < 0.005).sum())
    # every output row is complete; the count is N + clones + splits - low-opacity prunes (low
    # opacity rows include clones / split children of low-opacity parents)
    n = out["xyz"].shape[0]
    assert all(v.shape[0] == n for v in out.values())
    assert n <= 500 + n_clone + n_split
    assert n >= 500 + n_clone + n_split - 3 * n_low
    # moments of appended rows are zero, statistics were reset
    assert float(out["grad_accum"].abs().sum()) == 0.0 and float(out["denom"].sum()) == 0.0
