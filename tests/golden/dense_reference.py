"""Independent dense torch restatement of the 3DGS forward (TEST INFRASTRUCTURE).

Every (pixel, Gaussian) pair is evaluated with plain tensor ops; gradients come from
torch autograd, not from a hand-written backward.  It shares no code with the CPU oracle
(oracle/gsr_oracle.c) or the HIP kernels, so agreement pins both hand-written backwards.

Spec: SURVEY.md Appendix B (B.1 preprocess, B.3 blend).  The discrete decisions (cull,
tile rect, depth order, power > 0, alpha < 1/255, T < 1e-4 termination) are evaluated in
float32 with the spec's operation order; values are carried in ``dtype`` (float64 for
the golden fixtures) so autograd gives reference gradients.
"""
from __future__ import annotations

import math

import torch

SH_C0 = 0.28209479177387814
SH_C1 = 0.4886025119029199
SH_C2 = [1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792,
         0.5462742152960396]
SH_C3 = [-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154,
         -0.4570457994644658, 1.445305721320277, -0.5900435899266435]


def sh_basis(D, x, y, z):
    b = [torch.full_like(x, SH_C0)]
    if D >= 1:
        b += [-SH_C1 * y, SH_C1 * z, -SH_C1 * x]
    if D >= 2:
        xx, yy, zz = x * x, y * y, z * z
        b += [SH_C2[0] * x * y, SH_C2[1] * y * z, SH_C2[2] * (2 * zz - xx - yy), SH_C2[3] * x * z,
              SH_C2[4] * (xx - yy)]
    if D >= 3:
        b += [SH_C3[0] * y * (3 * xx - yy), SH_C3[1] * x * y * z, SH_C3[2] * y * (4 * zz - xx - yy),
              SH_C3[3] * z * (2 * zz - 3 * xx - 3 * yy), SH_C3[4] * x * (4 * zz - xx - yy),
              SH_C3[5] * z * (xx - yy), SH_C3[6] * x * (xx - 3 * yy)]
    return torch.stack(b, dim=1)  # (P, nb)


def preprocess(cam, means, opac, scales=None, rots=None, sh_dc=None, sh_rest=None, D=0,
               colors=None, cov3D=None, scale_mod=1.0, dtype=torch.float64):
    """Differentiable preprocess.  Returns dict with xy (pixel), depth, conic (A,B,C),
    opacity, rgb, radius (int), rect, visible; plus the NDC hook tensor."""
    V = torch.tensor(cam.viewmatrix, dtype=dtype)
    Pm = torch.tensor(cam.projmatrix, dtype=dtype)
    x, y, z = means[:, 0], means[:, 1], means[:, 2]
    tx = V[0] * x + V[4] * y + V[8] * z + V[12]
    ty = V[1] * x + V[5] * y + V[9] * z + V[13]
    tz = V[2] * x + V[6] * y + V[10] * z + V[14]
    hx = Pm[0] * x + Pm[4] * y + Pm[8] * z + Pm[12]
    hy = Pm[1] * x + Pm[5] * y + Pm[9] * z + Pm[13]
    hw = Pm[3] * x + Pm[7] * y + Pm[11] * z + Pm[15]
    pw = 1.0 / (hw + 1e-7)
    ndc = torch.stack([hx * pw, hy * pw], dim=1)
    hook = torch.zeros_like(ndc, requires_grad=True)  # screen-space gradient probe
    ndc = ndc + hook
    if cov3D is None:
        r, qx, qy, qz = rots[:, 0], rots[:, 1], rots[:, 2], rots[:, 3]
        R = torch.stack([
            1 - 2 * (qy * qy + qz * qz), 2 * (qx * qy - r * qz), 2 * (qx * qz + r * qy),
            2 * (qx * qy + r * qz), 1 - 2 * (qx * qx + qz * qz), 2 * (qy * qz - r * qx),
            2 * (qx * qz - r * qy), 2 * (qy * qz + r * qx), 1 - 2 * (qx * qx + qy * qy)],
            dim=1).reshape(-1, 3, 3)
        L = R * (scale_mod * scales)[:, None, :]
        S = L @ L.transpose(1, 2)
    else:
        c = cov3D
        S = torch.stack([c[:, 0], c[:, 1], c[:, 2], c[:, 1], c[:, 3], c[:, 4], c[:, 2], c[:, 4], c[:, 5]],
                        dim=1).reshape(-1, 3, 3)
    W, H = cam.width, cam.height
    fx = W / (2.0 * cam.tanfovx)
    fy = H / (2.0 * cam.tanfovy)
    limx, limy = 1.3 * cam.tanfovx, 1.3 * cam.tanfovy
    cx = torch.clamp(tx / tz, -limx, limx) * tz
    cy = torch.clamp(ty / tz, -limy, limy) * tz
    zero = torch.zeros_like(tz)
    J = torch.stack([fx / tz, zero, -(fx * cx) / (tz * tz), zero, fy / tz, -(fy * cy) / (tz * tz)],
                    dim=1).reshape(-1, 2, 3)
    Wv = torch.stack([V[0], V[4], V[8], V[1], V[5], V[9], V[2], V[6], V[10]]).reshape(3, 3)
    T = J @ Wv
    cov = T @ S @ T.transpose(1, 2)
    a = cov[:, 0, 0] + 0.3
    b = cov[:, 0, 1]
    c2 = cov[:, 1, 1] + 0.3
    det = a * c2 - b * b
    conic = torch.stack([c2 / det, -b / det, a / det], dim=1)
    xy = torch.stack([((ndc[:, 0] + 1.0) * W - 1.0) * 0.5, ((ndc[:, 1] + 1.0) * H - 1.0) * 0.5], dim=1)
    if colors is None:
        dv = means - torch.tensor(cam.campos, dtype=dtype)
        dirs = dv / torch.sqrt((dv * dv).sum(1, keepdim=True))
        basis = sh_basis(D, dirs[:, 0], dirs[:, 1], dirs[:, 2])  # (P, nb)
        nb = (D + 1) ** 2
        coeffs = sh_dc if nb == 1 else torch.cat([sh_dc, sh_rest[:, :nb - 1]], dim=1)  # (P,nb,3)
        res = (basis[:, :, None] * coeffs).sum(1) + 0.5
        rgb = torch.clamp_min(res, 0.0)
    else:
        rgb = colors
    return dict(xy=xy, depth=tz, conic=conic, opacity=opac.reshape(-1), rgb=rgb, hook=hook,
                a=a, b=b, c=c2, det=det, tz=tz)


def geometry_f32(cam, means, opac, scales=None, rots=None, cov3D=None, scale_mod=1.0):
    """Non-differentiable discrete decisions in float32 (spec op order): radius, rect,
    visibility.  Must agree bit-for-bit with the oracle's radii."""
    with torch.no_grad():
        f = lambda a: None if a is None else torch.as_tensor(a, dtype=torch.float32)
        V = torch.tensor(cam.viewmatrix, dtype=torch.float32)
        Pm = torch.tensor(cam.projmatrix, dtype=torch.float32)
        m = f(means)
        x, y, z = m[:, 0], m[:, 1], m[:, 2]
        tx = V[0] * x + V[4] * y + V[8] * z + V[12]
        ty = V[1] * x + V[5] * y + V[9] * z + V[13]
        tz = V[2] * x + V[6] * y + V[10] * z + V[14]
        hx = Pm[0] * x + Pm[4] * y + Pm[8] * z + Pm[12]
        hy = Pm[1] * x + Pm[5] * y + Pm[9] * z + Pm[13]
        hw = Pm[3] * x + Pm[7] * y + Pm[11] * z + Pm[15]
        pw = torch.tensor(1.0, dtype=torch.float32) / (hw + torch.tensor(1e-7, dtype=torch.float32))
        px, py = hx * pw, hy * pw
        if cov3D is None:
            q = f(rots)
            r, qx, qy, qz = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
            one, two = torch.tensor(1.0), torch.tensor(2.0)
            R = [one - two * (qy * qy + qz * qz), two * (qx * qy - r * qz), two * (qx * qz + r * qy),
                 two * (qx * qy + r * qz), one - two * (qx * qx + qz * qz), two * (qy * qz - r * qx),
                 two * (qx * qz - r * qy), two * (qy * qz + r * qx), one - two * (qx * qx + qy * qy)]
            s = f(scales) * torch.tensor(scale_mod, dtype=torch.float32)
            L = [R[3 * i + j] * s[:, j] for i in range(3) for j in range(3)]
            sig = lambda i, j: L[3 * i] * L[3 * j] + L[3 * i + 1] * L[3 * j + 1] + L[3 * i + 2] * L[3 * j + 2]
            c3 = [sig(0, 0), sig(0, 1), sig(0, 2), sig(1, 1), sig(1, 2), sig(2, 2)]
        else:
            cc = f(cov3D)
            c3 = [cc[:, k] for k in range(6)]
        W, H = cam.width, cam.height
        Wf, Hf = torch.tensor(float(W)), torch.tensor(float(H))
        tfx, tfy = torch.tensor(cam.tanfovx, dtype=torch.float32), torch.tensor(cam.tanfovy, dtype=torch.float32)
        fx = Wf / (torch.tensor(2.0) * tfx)
        fy = Hf / (torch.tensor(2.0) * tfy)
        limx, limy = torch.tensor(1.3) * tfx, torch.tensor(1.3) * tfy
        cx = torch.minimum(limx, torch.maximum(-limx, tx / tz)) * tz
        cy = torch.minimum(limy, torch.maximum(-limy, ty / tz)) * tz
        tz2 = tz * tz
        J00, J02 = fx / tz, -(fx * cx) / tz2
        J11, J12 = fy / tz, -(fy * cy) / tz2
        T0 = [J00 * V[4 * k + 0] + J02 * V[4 * k + 2] for k in range(3)]
        T1 = [J11 * V[4 * k + 1] + J12 * V[4 * k + 2] for k in range(3)]
        S = [c3[0], c3[1], c3[2], c3[1], c3[3], c3[4], c3[2], c3[4], c3[5]]
        U0 = [T0[0] * S[j] + T0[1] * S[3 + j] + T0[2] * S[6 + j] for j in range(3)]
        U1 = [T1[0] * S[j] + T1[1] * S[3 + j] + T1[2] * S[6 + j] for j in range(3)]
        a = (U0[0] * T0[0] + U0[1] * T0[1] + U0[2] * T0[2]) + torch.tensor(0.3)
        b = U0[0] * T1[0] + U0[1] * T1[1] + U0[2] * T1[2]
        c = (U1[0] * T1[0] + U1[1] * T1[1] + U1[2] * T1[2]) + torch.tensor(0.3)
        det = a * c - b * b
        mid = torch.tensor(0.5) * (a + c)
        disc = torch.maximum(torch.tensor(0.1), mid * mid - det)
        sq = torch.sqrt(disc)
        lam = torch.maximum(mid + sq, mid - sq)
        radius = torch.ceil(torch.tensor(3.0) * torch.sqrt(lam)).to(torch.int32)
        xs = ((px + 1.0) * Wf - 1.0) * 0.5
        ys = ((py + 1.0) * Hf - 1.0) * 0.5
        gx, gy = (W + 15) // 16, (H + 15) // 16
        rf = radius.to(torch.float32)
        t16 = torch.tensor(16.0)
        rect = torch.stack([
            torch.clamp(torch.trunc((xs - rf) / t16).to(torch.int64), 0, gx),
            torch.clamp(torch.trunc((ys - rf) / t16).to(torch.int64), 0, gy),
            torch.clamp(torch.trunc((xs + rf + 15.0) / t16).to(torch.int64), 0, gx),
            torch.clamp(torch.trunc((ys + rf + 15.0) / t16).to(torch.int64), 0, gy)], dim=1)
        area = (rect[:, 2] - rect[:, 0]) * (rect[:, 3] - rect[:, 1])
        visible = (tz > 0.2) & (det != 0) & (area > 0)
        radius = torch.where(visible, radius, torch.zeros_like(radius))
        return dict(radius=radius, rect=rect, visible=visible, depth=tz)


def render(cam, pre, geom, bg, gid_order=None):
    """Dense front-to-back compositing over every pixel, Gaussians in (depth_bits, gid)
    order, restricted to pixels whose tile lies in the Gaussian's rect."""
    dtype = pre["xy"].dtype
    W, H = cam.width, cam.height
    vis = geom["visible"]
    depth32 = geom["depth"].to(torch.float32)
    bits = depth32.view(torch.int32).to(torch.int64)
    idx = torch.nonzero(vis).reshape(-1)
    order = idx[torch.argsort(bits[idx] * (1 << 32) + idx, stable=True)]
    py, px = torch.meshgrid(torch.arange(H), torch.arange(W), indexing="ij")
    pfx, pfy = px.reshape(-1).to(dtype), py.reshape(-1).to(dtype)
    tile_x, tile_y = px.reshape(-1) // 16, py.reshape(-1) // 16
    npx = H * W
    T = torch.ones(npx, dtype=dtype)
    C = torch.zeros(3, npx, dtype=dtype)
    alive = torch.ones(npx, dtype=torch.bool)
    last = torch.zeros(npx, dtype=torch.int64)
    contributor = torch.zeros(npx, dtype=torch.int64)
    T32 = torch.ones(npx, dtype=torch.float32)
    for g in order.tolist():
        r = geom["rect"][g]
        inr = (tile_x >= r[0]) & (tile_x < r[2]) & (tile_y >= r[1]) & (tile_y < r[3])
        contributor = contributor + (inr & alive).to(torch.int64)
        dx = pre["xy"][g, 0] - pfx
        dy = pre["xy"][g, 1] - pfy
        co = pre["conic"][g]
        power = -0.5 * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy
        Gv = torch.exp(power)
        alpha = torch.clamp_max(pre["opacity"][g] * Gv, 0.99)
        with torch.no_grad():
            a32 = alpha.to(torch.float32)
            keep = inr & alive & (power.to(torch.float32) <= 0) & (a32 >= 1.0 / 255.0)
            test32 = T32 * (1.0 - a32)
            term = keep & (test32 < 1e-4)
            alive = alive & ~term
            keep = keep & ~term
            T32 = torch.where(keep, test32, T32)
            last = torch.where(keep, contributor, last)
        w = torch.where(keep, alpha * T, torch.zeros_like(T))
        C = C + pre["rgb"][g][:, None] * w[None, :]
        T = torch.where(keep, T * (1.0 - alpha), T)
    bgt = torch.as_tensor(bg, dtype=dtype)
    out = C + T[None, :] * bgt[:, None]
    return out.reshape(3, H, W), T.reshape(H, W), last.reshape(H, W)
