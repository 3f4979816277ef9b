"""TEST INFRASTRUCTURE ONLY -- CPU restatements of the training-step pieces around the
rasterizer.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module; the product (3d_gaussian_splatting_amd/) never does.

* ``ssim_loss``    the photometric loss (1 - lambda) L1 + lambda (1 - SSIM) as torch conv2d
                   code (upstream 3DGS utils/loss_utils: gaussian(11, 1.5) window built in
                   f64 then stored f32, zero padding 5, C1 = 0.01^2, C2 = 0.03^2, mean over
                   C x H x W); gradients by autograd.  The reference has no loss code (its
                   loop, src/utils/train_utils.cpp:128-145, is a stub): parity against the
                   reference itself is unpinned; this restatement is cross-checked against
                   closed forms and finite differences (tests/test_train_oracle.py).
* ``adam_step``    libtorch's torch::optim::Adam step (amsgrad off, weight_decay 0) in numpy
                   f32, the optimizer the reference builds (src/scene/gaussian_model.cpp:
                   323-345, default AdamOptions); pinned against torch.optim.Adam.
* ``raw_grads``    the getters' activation backward (exp / sigmoid / F.normalize,
                   src/scene/gaussian_model.cpp:54-58,270-298) by torch autograd.
* ``densify_and_prune``  upstream densify_and_clone / densify_and_split / prune_points on plain
                   CPU tensors with caller-given split samples (the reference only declares
                   the statistics tensors, src/scene/gaussian_model.h:18-20).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F


# ------------------------------------------------------------------------------- loss
def gaussian_window(size: int = 11, sigma: float = 1.5) -> torch.Tensor:
    g = torch.tensor([math.exp(-(x - size // 2) ** 2 / float(2 * sigma ** 2)) for x in range(size)],
                     dtype=torch.float32)
    return g / g.sum()


def ssim(img1: torch.Tensor, img2: torch.Tensor, window_size: int = 11) -> torch.Tensor:
    """Mean SSIM of two (C, H, W) images (upstream _ssim with size_average)."""
    C = img1.shape[-3]
    g = gaussian_window(window_size).to(img1.dtype).unsqueeze(1)
    w2 = g.mm(g.t()).unsqueeze(0).unsqueeze(0)
    window = w2.expand(C, 1, window_size, window_size).contiguous()
    x, y = img1.unsqueeze(0), img2.unsqueeze(0)
    pad = window_size // 2
    mu1 = F.conv2d(x, window, padding=pad, groups=C)
    mu2 = F.conv2d(y, window, padding=pad, groups=C)
    mu1_sq, mu2_sq, mu1_mu2 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    sigma1_sq = F.conv2d(x * x, window, padding=pad, groups=C) - mu1_sq
    sigma2_sq = F.conv2d(y * y, window, padding=pad, groups=C) - mu2_sq
    sigma12 = F.conv2d(x * y, window, padding=pad, groups=C) - mu1_mu2
    C1, C2 = 0.01 ** 2, 0.03 ** 2
    ssim_map = ((2 * mu1_mu2 + C1) * (2 * sigma12 + C2)) / ((mu1_sq + mu2_sq + C1) * (sigma1_sq + sigma2_sq + C2))
    return ssim_map.mean()


def ssim_loss(img, gt, lambda_dssim: float = 0.2, dtype=torch.float32):
    """-> (loss, l1, ssim, dL/dimg) as numpy (float64 scalars, dtype array)."""
    x = torch.as_tensor(np.asarray(img)).to(dtype).requires_grad_(True)
    y = torch.as_tensor(np.asarray(gt)).to(dtype)
    l1 = (x - y).abs().mean()
    s = ssim(x, y)
    loss = (1.0 - lambda_dssim) * l1 + lambda_dssim * (1.0 - s)
    loss.backward()
    return float(loss.detach()), float(l1.detach()), float(s.detach()), x.grad.numpy()


# ------------------------------------------------------------------------------- Adam
def adam_step(p, g, m, v, step: int, lr: float, beta1=0.9, beta2=0.999, eps=1e-8):
    """libtorch torch::optim::Adam::step for one parameter (torch/csrc/api/src/optim/adam.cpp):
      exp_avg.mul_(beta1).add_(grad, 1 - beta1)
      exp_avg_sq.mul_(beta2).addcmul_(grad, grad, 1 - beta2)
      denom = (exp_avg_sq.sqrt() / sqrt(bias_correction2)).add_(eps)
      param.addcdiv_(exp_avg, denom, -lr / bias_correction1)
    bias corrections in double, scalars cast to f32.  In-place on f32 numpy arrays."""
    f = np.float32
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    m *= f(beta1)
    m += f(1.0 - beta1) * g
    v *= f(beta2)
    v += f(1.0 - beta2) * g * g
    denom = np.sqrt(v) / f(math.sqrt(bc2)) + f(eps)
    p += f(-lr / bc1) * (m / denom)
    return p, m, v


def raw_grads(scaling_raw, rotation_raw, opacity_raw, d_scales, d_rots, d_opac):
    """Gradients w.r.t. the raw leaves given gradients w.r.t. the activated values
    (exp / F.normalize / sigmoid), by torch autograd in f32."""
    s = torch.as_tensor(np.asarray(scaling_raw, np.float32)).requires_grad_(True)
    q = torch.as_tensor(np.asarray(rotation_raw, np.float32)).requires_grad_(True)
    o = torch.as_tensor(np.asarray(opacity_raw, np.float32)).requires_grad_(True)
    out = (torch.exp(s) * torch.as_tensor(np.asarray(d_scales, np.float32))).sum() + \
        (F.normalize(q, p=2, dim=1) * torch.as_tensor(np.asarray(d_rots, np.float32))).sum() + \
        (torch.sigmoid(o) * torch.as_tensor(np.asarray(d_opac, np.float32))).sum()
    out.backward()
    return s.grad.numpy(), q.grad.numpy(), o.grad.numpy()


def activate(scaling_raw, rotation_raw, opacity_raw):
    s = torch.exp(torch.as_tensor(np.asarray(scaling_raw, np.float32)))
    q = F.normalize(torch.as_tensor(np.asarray(rotation_raw, np.float32)), p=2, dim=1)
    o = torch.sigmoid(torch.as_tensor(np.asarray(opacity_raw, np.float32)))
    return s.numpy(), q.numpy(), o.numpy()


# ------------------------------------------------------------------------------- densification
GROUPS = ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation")


def _build_rotation(r):
    norm = torch.sqrt(r[:, 0] * r[:, 0] + r[:, 1] * r[:, 1] + r[:, 2] * r[:, 2] + r[:, 3] * r[:, 3])
    q = r / norm[:, None]
    w, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R = torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
                     2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
                     2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)], dim=1)
    return R.reshape(-1, 3, 3)


def densify_and_prune(state: dict, max_grad: float, min_opacity: float, extent: float, max_screen_size,
                      percent_dense: float, split_samples: torch.Tensor) -> dict:
    """Upstream GaussianModel.densify_and_prune on a dict of CPU tensors:
    params (GROUPS), m_<g> / v_<g> Adam moments, grad_accum, denom, max_radii2D (all (N, ...)).
    Returns the new state dict."""
    st = {k: v.clone() for k, v in state.items()}

    def postfix(new):
        for g in GROUPS:
            st[g] = torch.cat([st[g], new[g]], 0)
            st["m_" + g] = torch.cat([st["m_" + g], torch.zeros_like(new[g])], 0)
            st["v_" + g] = torch.cat([st["v_" + g], torch.zeros_like(new[g])], 0)
        n = st["xyz"].shape[0]
        st["grad_accum"], st["denom"], st["max_radii2D"] = torch.zeros(n), torch.zeros(n), torch.zeros(n)

    def prune(mask):
        keep = ~mask
        for k in list(st.keys()):
            st[k] = st[k][keep]

    grads = state["grad_accum"] / state["denom"]
    grads[grads.isnan()] = 0.0
    # clone
    scaling = torch.exp(st["scaling"])
    sel = (grads >= max_grad) & (scaling.max(dim=1).values <= percent_dense * extent)
    postfix({g: st[g][sel] for g in GROUPS})
    # split (N = 2)
    n_init = st["xyz"].shape[0]
    padded = torch.zeros(n_init)
    padded[: grads.shape[0]] = grads
    scaling = torch.exp(st["scaling"])
    sel = (padded >= max_grad) & (scaling.max(dim=1).values > percent_dense * extent)
    N = 2
    rots = _build_rotation(st["rotation"][sel]).repeat(N, 1, 1)
    new = {"xyz": torch.bmm(rots, split_samples.unsqueeze(-1)).squeeze(-1) + st["xyz"][sel].repeat(N, 1),
           "scaling": torch.log(torch.exp(st["scaling"][sel]).repeat(N, 1) / (0.8 * N)),
           "rotation": st["rotation"][sel].repeat(N, 1), "f_dc": st["f_dc"][sel].repeat(N, 1, 1),
           "f_rest": st["f_rest"][sel].repeat(N, 1, 1), "opacity": st["opacity"][sel].repeat(N, 1)}
    postfix(new)
    prune(torch.cat([sel, torch.zeros(N * int(sel.sum()), dtype=torch.bool)]))
    # prune
    mask = (torch.sigmoid(st["opacity"]) < min_opacity).squeeze(1)
    if max_screen_size:
        mask = mask | (st["max_radii2D"] > max_screen_size) | (torch.exp(st["scaling"]).max(dim=1).values > 0.1 * extent)
    prune(mask)
    return st


def split_count(state: dict, max_grad: float, extent: float, percent_dense: float) -> int:
    """Number of Gaussians densify_and_split will split (so tests can draw its samples)."""
    grads = state["grad_accum"] / state["denom"]
    grads[grads.isnan()] = 0.0
    scaling = torch.exp(state["scaling"])
    clone = (grads >= max_grad) & (scaling.max(dim=1).values <= percent_dense * extent)
    split = (grads >= max_grad) & (scaling.max(dim=1).values > percent_dense * extent)
    del clone
    return int(split.sum())
