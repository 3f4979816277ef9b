"""The training loop (BASELINE configs[4]): the reference's ``train()`` loop,
src/utils/train_utils.cpp:128-145, with the body its stub leaves out, on a synthetic
Mip-NeRF360-scale scene.

Per iteration, in the reference's order (``GaussianTrainer.step``): xyz learning-rate update,
SH degree +1 every 1000 iterations, a camera popped from a shuffled stack of the training
views (refilled when empty, as upstream), render -> L1 + D-SSIM loss -> backward, densification
statistics, densify / prune every ``densification_interval`` iterations in
[``densify_from_iter``, ``densify_until_iter``), opacity reset every ``opacity_reset_interval``,
then the fused Adam step -- with the OptimizationParams defaults of src/arguments/params.h:50-91.
No host synchronisation inside an iteration except the densification read-backs; the loss is
read back only at the log points.

The scene: ground-truth images rendered by the same rasterizer from a procedural cloud of
Gaussians (a textured ground disc and a few object blobs, SH degree 1) seen by cameras on an
orbit around it -- the shape of a Mip-NeRF360 capture (a few hundred views of an unbounded
scene around a central object) with no dataset to download; training starts from a sparse,
noisy sample of the ground-truth centres and colours (the upstream create_from_pcd path).
"""
from __future__ import annotations

import math
import sys
import time
from dataclasses import dataclass, field

import numpy as np
import torch

from . import graphics
from .rasterizer import CAbiRasterizer
from .scene import normal, uniform
from .trainer import GaussianTrainer, OptimizationParams


@dataclass
class LoopScene:
    cams: list
    gts: list            # (3, H, W) f32 device tensors in [0, 1]
    points: np.ndarray   # (n, 3) initial point cloud
    colors: np.ndarray   # (n, 3) its colours in [0, 1]
    extent: float        # camera extent (nerf++ radius), spatial_lr_scale upstream
    n_gt: int = 0


def look_at_camera(center, target, fovx: float, width: int, height: int) -> graphics.RasterCamera:
    """A camera at `center` looking at `target` (COLMAP axes: x right, y down, z forward),
    built through graphics.make_camera like the reference's Camera (camera.cpp:66-71)."""
    c = np.asarray(center, np.float64)
    f = np.asarray(target, np.float64) - c
    f /= np.linalg.norm(f)
    d = np.array([0.0, 1.0, 0.0])
    y = d - f * (d @ f)
    y /= np.linalg.norm(y)
    x = np.cross(y, f)
    Rt = np.stack([x, y, f])  # world -> camera rows
    R = Rt.T
    t = -Rt @ c
    fovy = 2.0 * math.atan(math.tan(fovx / 2.0) * height / width)
    return graphics.make_camera(R, t, fovx, fovy, width, height)


def orbit_cameras(n_views: int, width: int, height: int, radius: float = 4.0, seed: int = 0,
                  fovx_deg: float = 60.0) -> list:
    """Views on a ring around the origin (heights and radii jittered), all looking at it."""
    u = uniform(seed, 11, 3 * n_views).reshape(n_views, 3)
    cams = []
    for i in range(n_views):
        a = 2.0 * math.pi * (i + 0.5 * u[i, 0]) / n_views
        r = radius * (0.9 + 0.2 * u[i, 1])
        h = -1.2 + 0.8 * u[i, 2]  # y points down: cameras slightly above the ground disc
        cams.append(look_at_camera((r * math.sin(a), h, r * math.cos(a)), (0.0, 0.2, 0.0), math.radians(fovx_deg),
                                   width, height))
    return cams


def procedural_cloud(n: int, seed: int = 0, texture: float = 0.25, gt_scale: float = 0.012):
    """Ground-truth Gaussians: 60 % a textured ground disc (radius 3, y = 0.6), 40 % in five
    ellipsoidal blobs above it.  Returns raw leaves (means, f_dc, f_rest (SH1), opacity logits,
    log scales, quaternions) as numpy arrays."""
    u = uniform(seed, 21, 4 * n).reshape(n, 4)
    nz = normal(seed, 22, 3 * n).reshape(n, 3)
    n_ground = int(0.6 * n)
    means = np.zeros((n, 3))
    r = 3.0 * np.sqrt(u[:n_ground, 0])
    th = 2.0 * math.pi * u[:n_ground, 1]
    means[:n_ground] = np.stack([r * np.cos(th), 0.6 + 0.01 * nz[:n_ground, 0], r * np.sin(th)], 1)
    centres = np.array([[0.0, 0.1, 0.0], [0.9, 0.3, 0.4], [-0.8, 0.25, -0.5], [0.3, 0.35, -1.0], [-0.4, 0.3, 1.0]])
    radii = np.array([[0.45, 0.5, 0.45], [0.25, 0.3, 0.25], [0.3, 0.35, 0.2], [0.2, 0.25, 0.3], [0.3, 0.3, 0.3]])
    k = (u[n_ground:, 2] * len(centres)).astype(int)
    means[n_ground:] = centres[k] + radii[k] * nz[n_ground:] * 0.6
    # colours: smooth functions of position (checker-ish ground, tinted blobs)
    p = means
    base = np.stack([0.5 + 0.4 * np.sin(3.0 * p[:, 0]) * np.cos(3.0 * p[:, 2]),
                     0.5 + 0.35 * np.cos(2.0 * p[:, 0] + 1.0),
                     0.5 + 0.3 * np.sin(2.5 * p[:, 2] - 0.5)], 1)
    base[n_ground:] = 0.5 * base[n_ground:] + 0.5 * np.array([[0.9, 0.3, 0.2], [0.2, 0.7, 0.3], [0.2, 0.3, 0.9],
                                                              [0.8, 0.8, 0.2], [0.7, 0.2, 0.8]])[k]
    # per-splat colour noise: fine texture (a captured scene's high-frequency detail, which is
    # what drives densification -- a smooth cloud is fitted by few Gaussians)
    base = base + texture * normal(seed, 27, 3 * n).reshape(n, 3)
    f_dc = ((np.clip(base, 0.02, 0.98) - 0.5) / 0.28209479177387814)[:, None, :]
    f_rest = 0.05 * normal(seed, 23, 9 * n).reshape(n, 3, 3)
    log_s = np.log(gt_scale) + 0.4 * normal(seed, 24, 3 * n).reshape(n, 3)
    log_s[:n_ground, 1] = np.log(0.002)  # flat ground splats
    q = normal(seed, 25, 4 * n).reshape(n, 4)
    q[:n_ground] = [1.0, 0.0, 0.0, 0.0]
    opac = 1.5 + 0.8 * normal(seed, 26, n)[:, None]
    f32 = lambda a: np.ascontiguousarray(a, dtype=np.float32)
    return f32(means), f32(f_dc), f32(f_rest), f32(opac), f32(log_s), f32(q), f32(np.clip(base, 0, 1))


def synthetic_scene(n_gt: int, n_init: int, n_views: int, width: int, height: int, seed: int = 0,
                    device="cuda", texture: float = 0.25, gt_scale: float = 0.012) -> LoopScene:
    """Ground truth rendered once per view (the rasterizer's forward, no gradients), and a
    sparse noisy initial point cloud."""
    means, f_dc, f_rest, opac, log_s, q, rgb = procedural_cloud(n_gt, seed, texture, gt_scale)
    cams = orbit_cameras(n_views, width, height, seed=seed)
    dev = torch.device(device)
    t = lambda a: torch.as_tensor(a, device=dev)
    sc, qq = torch.exp(t(log_s)), torch.nn.functional.normalize(t(q), dim=1)
    op = torch.sigmoid(t(opac)).reshape(-1)
    rast = CAbiRasterizer(dev)
    gts = []
    for cam in cams:
        st = rast.forward(cam, t(means), op, scales=sc, rotations=qq, sh_dc=t(f_dc), sh_rest=t(f_rest), sh_degree=1)
        gts.append(st.color.clamp(0.0, 1.0).contiguous())
    pick = (uniform(seed, 31, n_init) * n_gt).astype(np.int64)
    pts = means[pick] + 0.02 * normal(seed, 32, 3 * n_init).reshape(n_init, 3).astype(np.float32)
    centres = np.stack([c.campos for c in cams]).astype(np.float64)
    extent = float(np.linalg.norm(centres - centres.mean(0), axis=1).max() * 1.1)  # get_nerfpp_norm radius
    return LoopScene(cams=cams, gts=gts, points=pts.astype(np.float32), colors=rgb[pick], extent=extent, n_gt=n_gt)


@dataclass
class LoopResult:
    iterations: int
    seconds: float
    iters_per_s: float
    num_points: list = field(default_factory=list)  # (iteration, count) after each densification
    loss: list = field(default_factory=list)        # (iteration, loss, l1, ssim) at the log points
    final_points: int = 0
    peak_points: int = 0
    binning_overflows: int = 0   # bounded renders whose K exceeded the bound (must stay 0)
    exact_k_reads: int = 0       # renders sized by a host read of K (after each point-set change)


def view_sequence(n_views: int, iterations: int, seed: int = 0) -> np.ndarray:
    """The camera of each iteration: the viewpoint stack refilled with a random permutation of
    the training views whenever it runs empty and popped from its end, as upstream."""
    rng = np.random.default_rng(seed)
    stack: list = []
    out = np.empty(iterations, np.int32)
    for i in range(iterations):
        if not stack:
            stack = list(rng.permutation(n_views))
        out[i] = int(stack.pop())
    return out


def write_scene(path: str, scene: LoopScene, iterations: int, opt: OptimizationParams | None = None,
                max_sh_degree: int = 3, seed: int = 0, log_every: int = 100, densify: bool = True,
                progress_every: int = 0, views=None) -> None:
    """The GSRLOOP1 file tests/cpp/train_main.cpp (lib/gsr_train_loop) reads: the scene, the
    OptimizationParams (as the reference's float fields) and the camera of every iteration."""
    opt = opt or OptimizationParams()
    views = view_sequence(len(scene.cams), iterations, seed) if views is None else np.asarray(views, np.int32)
    H, W = int(scene.gts[0].shape[1]), int(scene.gts[0].shape[2])
    with open(path, "wb") as f:
        f.write(b"GSRLOOP1")
        f.write(np.array([len(scene.cams), W, H, len(scene.points), iterations, max_sh_degree, seed, log_every,
                          int(densify), progress_every], np.int32).tobytes())
        f.write(np.array([opt.iterations, opt.position_lr_max_steps, opt.densification_interval,
                          opt.opacity_reset_interval, opt.densify_from_iter, opt.densify_until_iter,
                          int(opt.random_background)], np.int32).tobytes())
        f.write(np.array([opt.position_lr_init, opt.position_lr_final, opt.position_lr_delay_mult, opt.feature_lr,
                          opt.opacity_lr, opt.scaling_lr, opt.rotation_lr, opt.percent_dense, opt.lambda_dssim,
                          opt.densify_grad_threshold], np.float32).tobytes())
        f.write(np.array([scene.extent], np.float64).tobytes())
        f.write(np.zeros(3, np.float32).tobytes())  # black background (train_utils.cpp:115-116)
        for c in scene.cams:
            f.write(np.concatenate([[c.tanfovx, c.tanfovy], np.asarray(c.viewmatrix, np.float32).ravel(),
                                    np.asarray(c.projmatrix, np.float32).ravel(),
                                    np.asarray(c.campos, np.float32).ravel()]).astype(np.float32).tobytes())
        for g in scene.gts:
            f.write(g.detach().cpu().numpy().astype(np.float32).tobytes())
        f.write(np.ascontiguousarray(scene.points, np.float32).tobytes())
        f.write(np.ascontiguousarray(scene.colors, np.float32).tobytes())
        f.write(views.astype(np.int32).tobytes())


def train(scene: LoopScene, iterations: int | None = None, opt: OptimizationParams | None = None,
          max_sh_degree: int = 3, seed: int = 0, log_every: int = 100, device="cuda",
          progress_every: int = 0) -> LoopResult:
    """train_utils.cpp:128-145 over `scene` (GaussianTrainer.from_point_cloud = create_from_pcd,
    spatial_lr_scale = the camera extent).  progress_every > 0 prints a line to stderr every
    that many iterations (no device sync)."""
    opt = opt or OptimizationParams()
    iterations = iterations or opt.iterations
    tr = GaussianTrainer.from_point_cloud(scene.points, scene.colors, max_sh_degree, spatial_lr_scale=scene.extent,
                                          opt=opt, device=device, seed=seed)
    views = view_sequence(len(scene.cams), iterations, seed)
    res = LoopResult(iterations=iterations, seconds=0.0, iters_per_s=0.0)
    logged = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for it in range(1, iterations + 1):
        v = int(views[it - 1])
        out = tr.step(it, scene.cams[v], scene.gts[v])
        if it % log_every == 0 or it == 1 or it == iterations:
            logged.append((it, out["stats"]))
        if it < opt.densify_until_iter and it > opt.densify_from_iter and it % opt.densification_interval == 0:
            res.num_points.append((it, tr.num_points))
        res.peak_points = max(res.peak_points, tr.num_points)
        if progress_every and it % progress_every == 0:
            print(f"[loop] iteration {it} points {tr.num_points} {time.perf_counter() - t0:.1f} s", file=sys.stderr,
                  flush=True)
    torch.cuda.synchronize()
    res.seconds = time.perf_counter() - t0
    res.iters_per_s = iterations / res.seconds
    res.final_points = tr.num_points
    tr.binning.poll()
    res.binning_overflows = tr.binning.overflows
    res.exact_k_reads = tr.binning.exact_reads
    res.loss = [(it, *[float(x) for x in s.cpu().tolist()]) for it, s in logged]
    res.trainer = tr
    return res
