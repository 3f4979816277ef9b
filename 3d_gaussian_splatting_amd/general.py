"""Torch restatements of the reference's math utilities that sit on the rasterizer boundary.

  build_rotation          src/utils/general_utils.cpp:12-40   (q = (w,x,y,z), normalised first)
  strip_lowerdiag         src/utils/general_utils.cpp:49-62   ([xx,xy,xz,yy,yz,zz])
  strip_symmetric         src/utils/general_utils.cpp:73-76
  build_scaling_rotation  src/utils/general_utils.cpp:88-99   (L = R diag(s))
  build_covariance_from_scaling_rotation  src/scene/gaussian_model.cpp:18-28
  get_expon_lr_func       src/utils/general_utils.cpp:112-142 (used by the model's xyz LR)
  eval_sh                 SH basis of SURVEY Appendix B.1 (PipelineParams::convert_SHs_python_)

Device-agnostic (the reference hard-codes torch::kCUDA, general_utils.cpp:21,51,90).
"""
from __future__ import annotations

import math

import torch

SH_C0 = 0.28209479177387814
SH_C1 = 0.4886025119029199
SH_C2 = (1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792,
         0.5462742152960396)
SH_C3 = (-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154,
         -0.4570457994644658, 1.445305721320277, -0.5900435899266435)


def build_rotation(r: torch.Tensor) -> torch.Tensor:
    norm = torch.sqrt(r[:, 0] * r[:, 0] + r[:, 1] * r[:, 1] + r[:, 2] * r[:, 2] + r[:, 3] * r[:, 3])
    q = r / norm[:, None]
    rr, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R = torch.stack([
        1 - 2 * (y * y + z * z), 2 * (x * y - rr * z), 2 * (x * z + rr * y),
        2 * (x * y + rr * z), 1 - 2 * (x * x + z * z), 2 * (y * z - rr * x),
        2 * (x * z - rr * y), 2 * (y * z + rr * x), 1 - 2 * (x * x + y * y)], dim=1)
    return R.reshape(-1, 3, 3)


def strip_lowerdiag(L: torch.Tensor) -> torch.Tensor:
    return torch.stack([L[:, 0, 0], L[:, 0, 1], L[:, 0, 2], L[:, 1, 1], L[:, 1, 2], L[:, 2, 2]], dim=1)


def strip_symmetric(sym: torch.Tensor) -> torch.Tensor:
    return strip_lowerdiag(sym)


def build_scaling_rotation(s: torch.Tensor, r: torch.Tensor) -> torch.Tensor:
    L = torch.zeros((s.shape[0], 3, 3), dtype=s.dtype, device=s.device)
    L[:, 0, 0], L[:, 1, 1], L[:, 2, 2] = s[:, 0], s[:, 1], s[:, 2]
    return build_rotation(r) @ L


def build_covariance_from_scaling_rotation(scaling: torch.Tensor, scaling_modifier: float,
                                           rotation: torch.Tensor) -> torch.Tensor:
    L = build_scaling_rotation(scaling_modifier * scaling, rotation)
    return strip_symmetric(L @ L.transpose(1, 2))


def get_expon_lr_func(lr_init, lr_final, lr_delay_steps=0, lr_delay_mult=1.0, max_steps=1000000):
    def f(step):
        if step < 0 or (lr_init == 0.0 and lr_final == 0.0):
            return 0.0
        if lr_delay_steps > 0:
            delay_rate = lr_delay_mult + (1 - lr_delay_mult) * math.sin(
                0.5 * math.pi * min(max(step / lr_delay_steps, 0.0), 1.0))
        else:
            delay_rate = 1.0
        t = min(max(step / max_steps, 0.0), 1.0)
        return delay_rate * math.exp(math.log(lr_init) * (1 - t) + math.log(lr_final) * t)
    return f


def eval_sh(deg: int, sh: torch.Tensor, dirs: torch.Tensor) -> torch.Tensor:
    """sh: (P, M, 3), dirs: (P, 3) unit -> (P, 3) (without the +0.5 offset)."""
    res = SH_C0 * sh[:, 0]
    if deg > 0:
        x, y, z = dirs[:, 0:1], dirs[:, 1:2], dirs[:, 2:3]
        res = res - SH_C1 * y * sh[:, 1] + SH_C1 * z * sh[:, 2] - SH_C1 * x * sh[:, 3]
        if deg > 1:
            xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
            res = (res + SH_C2[0] * xy * sh[:, 4] + SH_C2[1] * yz * sh[:, 5] +
                   SH_C2[2] * (2.0 * zz - xx - yy) * sh[:, 6] + SH_C2[3] * xz * sh[:, 7] +
                   SH_C2[4] * (xx - yy) * sh[:, 8])
            if deg > 2:
                res = (res + SH_C3[0] * y * (3 * xx - yy) * sh[:, 9] + SH_C3[1] * xy * z * sh[:, 10] +
                       SH_C3[2] * y * (4 * zz - xx - yy) * sh[:, 11] +
                       SH_C3[3] * z * (2 * zz - 3 * xx - 3 * yy) * sh[:, 12] +
                       SH_C3[4] * x * (4 * zz - xx - yy) * sh[:, 13] + SH_C3[5] * z * (xx - yy) * sh[:, 14] +
                       SH_C3[6] * x * (xx - 3 * yy) * sh[:, 15])
    return res
