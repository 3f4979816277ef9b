"""Training step around the rasterizer, on the HIP kernels of
include/gsr/gsr_train.h.

What it mirrors in the reference (seiya-kumada/3d_gaussian_splatting):

* ``OptimizationParams``      src/arguments/params.h:50-91 (same fields and defaults).
* ``GaussianTrainer.setup``   GaussianModel::setup, src/scene/gaussian_model.cpp:316-352: six
  Adam instances with default AdamOptions (betas 0.9/0.999, eps 1e-8) and the xyz LR
  schedule.  The reference passes (init, final, delay_mult, max_steps) to a five-argument
  get_expon_lr_func (gaussian_model.cpp:347-351 against general_utils.h:8-13), which binds
  delay_mult to lr_delay_steps; the build calls it with the
  arguments the names say (delay_steps = 0, delay_mult, max_steps).
* ``update_learning_rate`` / ``oneup_SH_degree`` and the per-iteration order
  src/utils/train_utils.cpp:128-145 (LR update, SH degree +1 every 1000 iterations, render,
  loss, backward, statistics, densification, optimizer step).
* the statistics tensors ``max_radii2D_ / xyz_gradient_accum_ / denom_``
  (src/scene/gaussian_model.h:18-20; (N) here, not the reference's {1}-shaped accumulator,
  gaussian_model.cpp:319, Appendix A).
* densify_and_clone / densify_and_split / prune_points / reset_opacity: the upstream 3DGS
  semantics the reference's stats tensors exist for (the reference has no densification
  code).
* ``capture`` / ``restore``: GaussianModel::capture / restore (gaussian_model.cpp:76-267);
  ``from_point_cloud`` / ``save_ply`` / ``from_ply``: the upstream create_from_pcd / save_ply /
  load_ply, the k-NN scale initialisation on the GPU.

Device work per iteration, all through the C ABI: gsr_activate -> gsr_forward -> loss
forward/backward -> gsr_backward -> gsr_densify_stats -> gsr_adam_step (one launch for the
six groups, activation backward fused).  No host synchronisation inside ``step`` (the loss
stays on the device); densification (every ``densification_interval`` iterations) reads
counts back.  The forward's binning runs under a capacity bound (``BinningCapacity``), so K is
not read back either: the first render after a change in the point set is sized exactly (one
read of K), later ones by 1.5x the largest K seen, checked one iteration late from a pinned
copy.  No CPU fallback: the HIP library is required.
"""
from __future__ import annotations

import ctypes
import math
import warnings
from dataclasses import dataclass

import numpy as np
import torch

from . import native, scene_io
from .general import build_rotation, get_expon_lr_func
from .rasterizer import CAbiRasterizer

GROUPS = ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation")
ACTS = {"xyz": native.ACT_NONE, "f_dc": native.ACT_NONE, "f_rest": native.ACT_NONE,
        "opacity": native.ACT_SIGMOID, "scaling": native.ACT_EXP, "rotation": native.ACT_NORMALIZE4}


def _f32(x: float) -> float:
    return float(np.float32(x))


@dataclass
class OptimizationParams:
    """src/arguments/params.h:50-91.  The reference's fields are C++ float: the defaults here are
    those float values (so the C++ gsr::Trainer, which keeps the reference's struct, computes
    from the same numbers)."""
    iterations: int = 30_000
    position_lr_init: float = _f32(0.00016)
    position_lr_final: float = _f32(0.0000016)
    position_lr_delay_mult: float = _f32(0.01)
    position_lr_max_steps: int = 30_000
    feature_lr: float = _f32(0.0025)
    opacity_lr: float = _f32(0.05)
    scaling_lr: float = _f32(0.005)
    rotation_lr: float = _f32(0.001)
    percent_dense: float = _f32(0.01)
    lambda_dssim: float = _f32(0.2)
    densification_interval: int = 100
    opacity_reset_interval: int = 3000
    densify_from_iter: int = 500
    densify_until_iter: int = 15_000
    densify_grad_threshold: float = _f32(0.0002)
    random_background: bool = False


def _device(device) -> torch.device:
    d = torch.device(device)
    if d.type == "cuda" and d.index is None:
        d = torch.device("cuda", torch.cuda.current_device())
    return d


def _stream(dev):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


class TrainKernels:
    """ctypes front-end of include/gsr/gsr_train.h with torch-owned device memory."""

    def __init__(self, device="cuda"):
        self.device = _device(device)
        self.L = native.load_hip()

    def _check(self, rc, what):
        if rc != 0:
            raise RuntimeError(f"{what} failed ({rc}): {native.last_error()}")

    def activate(self, scale_raw, rot_raw, opac_raw):
        P = int(scale_raw.shape[0])
        s = torch.empty_like(scale_raw)
        q = torch.empty_like(rot_raw)
        o = torch.empty_like(opac_raw)
        self._check(self.L.gsr_activate(_p(scale_raw), _p(rot_raw), _p(opac_raw), P, _p(s), _p(q), _p(o),
                                        _stream(self.device)), "gsr_activate")
        return s, q, o

    def loss_forward(self, img, gt, lambda_dssim):
        """-> (stats (3,) device tensor [loss, l1, ssim], maps scratch for loss_backward)."""
        C, H, W = (int(v) for v in img.shape)
        if tuple(gt.shape) != (C, H, W):
            raise ValueError("loss: image / ground-truth shape mismatch")
        nbytes = int(self.L.gsr_loss_scratch_bytes(C, H, W))
        maps = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        stats = torch.empty(3, dtype=torch.float32, device=self.device)
        self._check(self.L.gsr_loss_forward(_p(img), _p(gt), C, H, W, float(lambda_dssim), _p(maps), _p(stats),
                                            _stream(self.device)), "gsr_loss_forward")
        return stats, maps

    def loss_backward(self, img, gt, lambda_dssim, maps):
        C, H, W = (int(v) for v in img.shape)
        out = torch.empty_like(img)
        self._check(self.L.gsr_loss_backward(_p(img), _p(gt), C, H, W, float(lambda_dssim), _p(maps), _p(out),
                                             _stream(self.device)), "gsr_loss_backward")
        return out

    def adam_step(self, groups, beta1=0.9, beta2=0.999, eps=1e-8, guard=None):
        """groups: list of dicts(param, grad, exp_avg, exp_avg_sq, act, step, lr), one launch.
        guard = (k_device, bound): the step is skipped on the device when the render's K
        exceeded the bound it ran under (gsr_adam_step_guarded)."""
        arr = (native.AdamGroup * len(groups))()
        for i, g in enumerate(groups):
            for k in ("param", "grad", "exp_avg", "exp_avg_sq"):
                t = g[k]
                if not (t.is_contiguous() and t.dtype == torch.float32 and t.device == self.device):
                    raise ValueError(f"adam: {k} must be a contiguous f32 tensor on {self.device}")
                if t.numel() != g["param"].numel():
                    raise ValueError(f"adam: {k} size mismatch")
                setattr(arr[i], k, t.data_ptr())
            arr[i].n = g["param"].numel()
            arr[i].act = int(g["act"])
            arr[i].step = int(g["step"])
            arr[i].lr = float(g["lr"])
        gk, gcap = _guard(guard)
        self._check(self.L.gsr_adam_step_guarded(arr, len(groups), float(beta1), float(beta2), float(eps), gk, gcap,
                                                 _stream(self.device)), "gsr_adam_step")

    def densify_stats(self, radii, dmeans2D, max_radii2D, grad_accum, denom, guard=None):
        P = int(radii.shape[0])
        gk, gcap = _guard(guard)
        self._check(self.L.gsr_densify_stats_guarded(_p(radii), _p(dmeans2D), P, _p(max_radii2D), _p(grad_accum),
                                                     _p(denom), gk, gcap, _stream(self.device)), "gsr_densify_stats")

    def compact_index(self, mask: torch.Tensor) -> torch.Tensor:
        """Ascending int32 indices of the nonzero entries of a bool / uint8 mask (one D2H read)."""
        m = mask.to(torch.uint8).contiguous()
        n = int(m.numel())
        idx = torch.empty(max(n, 1), dtype=torch.int32, device=self.device)
        cnt = torch.empty(1, dtype=torch.int32, device=self.device)
        scratch = torch.empty(int(self.L.gsr_compact_scratch_bytes(n)), dtype=torch.uint8, device=self.device)
        self._check(self.L.gsr_compact_index(_p(m), n, _p(idx), _p(cnt), _p(scratch), _stream(self.device)),
                    "gsr_compact_index")
        return idx[: int(cnt.item())]

    def knn_mean_dist2(self, points: torch.Tensor) -> torch.Tensor:
        """Mean squared distance of each point to its 3 nearest others (exact; gsr_knn_mean_dist2)."""
        if not (points.is_contiguous() and points.dtype == torch.float32 and points.device == self.device):
            raise ValueError(f"knn: points must be a contiguous f32 (N, 3) tensor on {self.device}")
        n = int(points.shape[0])
        out = torch.empty(n, dtype=torch.float32, device=self.device)
        if n == 0:
            return out
        scratch = torch.empty(int(self.L.gsr_knn_scratch_bytes(n)), dtype=torch.uint8, device=self.device)
        self._check(self.L.gsr_knn_mean_dist2(_p(points), n, _p(out), _p(scratch), _stream(self.device)),
                    "gsr_knn_mean_dist2")
        return out

    def gather_rows(self, tensors, idx: torch.Tensor):
        """[t[idx] for t in tensors] (rows) in one launch; tensors are (N, ...) f32."""
        n_out = int(idx.numel())
        outs = [torch.empty((n_out,) + tuple(t.shape[1:]), dtype=torch.float32, device=self.device)
                for t in tensors]
        if n_out == 0 or not tensors:
            return outs
        live = [i for i, t in enumerate(tensors) if math.prod(t.shape[1:]) > 0]  # skip (N, 0, 3) rows
        idx32 = idx.to(torch.int32).contiguous()
        for i0 in range(0, len(live), native.GATHER_MAX):
            chunk = live[i0:i0 + native.GATHER_MAX]
            arr = (native.RowCopy * len(chunk))()
            for j, i in enumerate(chunk):
                t = tensors[i]
                if not (t.is_contiguous() and t.dtype == torch.float32 and t.device == self.device):
                    raise ValueError("gather_rows: contiguous f32 device tensors only")
                arr[j].src, arr[j].dst = t.data_ptr(), outs[i].data_ptr()
                arr[j].width = int(math.prod(t.shape[1:]))
            self._check(self.L.gsr_gather_rows(arr, len(chunk), _p(idx32), n_out, _stream(self.device)),
                        "gsr_gather_rows")
        return outs


def _guard(guard):
    """(device pointer of K, bound) for the *_guarded entry points; (None, 0) = no guard."""
    if guard is None:
        return None, 0
    k, cap = guard
    return ctypes.c_void_p(k.data_ptr()), int(cap)


class BinningOverflowError(OverflowError):
    """A bounded render's K exceeded its bound (strict BinningCapacity): that render dropped
    instances, and the iteration that used it has been applied."""


class BinningCapacity:
    """max_rendered for the trainer's renders without a per-iteration host read of K.

    0 (exact sizing, the forward reads K back) right after the point set changes; afterwards
    ``headroom`` x the largest K seen, rounded up.  Each bounded render's K (the scan's device
    counter) is copied to a pinned slot and checked once its event has completed -- one or two
    iterations later, never waiting.  K above the bound at that check means that render was
    truncated (its kernels clamp to the bound; GSR_ERR_OVERFLOW semantics) and the iteration
    that used it has already run: its densification statistics and Adam step were skipped ON
    THE DEVICE (the trainer passes the render's K and bound to the *_guarded kernels, so a
    truncated render never updates the model), it is counted in ``overflows`` (with a warning
    the first time), the next render is sized exactly again, and with ``strict=True`` a
    BinningOverflowError is raised at that check instead.  The bound covers the largest K of
    the views rendered since the last point-set change with 1.5x + 64k headroom; views are
    re-rendered every len(views) iterations, so a view larger than that bound can only be one
    not yet seen since the change (the 30k-iteration loop: 0 overflows)."""

    def __init__(self, device, headroom: float = 1.5, ring: int = 8, strict: bool = False):
        self.headroom = float(headroom)
        self.strict = bool(strict)
        self.cap = 0
        self.k_max = 0
        self.overflows = 0
        self.exact_reads = 0
        pin = torch.cuda.is_available()
        self.slots = [torch.zeros(1, dtype=torch.int32, pin_memory=pin) for _ in range(ring)]
        self.pending: list = []  # (slot, event, cap)
        self.next_slot = 0

    def bound(self) -> int:
        self.poll()
        return self.cap

    def _grow(self):
        self.cap = (int(self.k_max * self.headroom) + 65536 + 4095) // 4096 * 4096

    def reset(self):
        """The point set changed: the next render is sized exactly."""
        self.pending.clear()
        self.cap = 0
        self.k_max = 0

    def observe(self, st):
        """After a forward: record its K (exact read, or an async copy under a bound)."""
        if self.cap == 0:
            self.exact_reads += 1
            self.k_max = max(self.k_max, st.num_rendered)
            self._grow()
            return
        if len(self.pending) == len(self.slots):
            self.pending[0][1].synchronize()
            self.poll()
        slot = self.slots[self.next_slot]
        self.next_slot = (self.next_slot + 1) % len(self.slots)
        slot.copy_(st.k_device(), non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(st.color.device))
        self.pending.append((slot, ev, self.cap))

    def poll(self):
        while self.pending and self.pending[0][1].query():
            slot, _, cap = self.pending.pop(0)
            k = int(slot.item())
            if k > cap:
                if self.overflows == 0:
                    warnings.warn(f"BinningCapacity: a render's K = {k} exceeded its bound {cap}; that iteration's "
                                  "update was skipped on the device and renders are sized exactly again",
                                  RuntimeWarning, stacklevel=2)
                self.overflows += 1
                self.k_max = max(self.k_max, k)
                self.pending.clear()
                self.cap = 0  # the next render is sized exactly
                if self.strict:
                    raise BinningOverflowError(f"a render's K = {k} exceeded its bound {cap}")
                return
            if k > self.k_max:
                self.k_max = k
                if k * 1.2 > self.cap:
                    self._grow()


class GaussianTrainer:
    """The reference GaussianModel's training state (raw leaves, Adam moments, statistics)
    with the per-iteration step on the HIP kernels."""

    def __init__(self, xyz, f_dc, f_rest, opacity, scaling, rotation, max_sh_degree: int,
                 opt: OptimizationParams | None = None, spatial_lr_scale: float = 1.0, device="cuda",
                 seed: int = 0, cameras_extent: float | None = None):
        self.device = _device(device)
        dev = self.device
        f = lambda a, shape: torch.as_tensor(a, dtype=torch.float32).reshape(shape).to(dev).contiguous()
        P = int(torch.as_tensor(xyz).shape[0])
        self.params = {"xyz": f(xyz, (P, 3)), "f_dc": f(f_dc, (P, 1, 3)),
                       "f_rest": f(f_rest, (P, -1, 3)), "opacity": f(opacity, (P, 1)),
                       "scaling": f(scaling, (P, 3)), "rotation": f(rotation, (P, 4))}
        self.max_sh_degree = int(max_sh_degree)
        self.active_sh_degree = 0
        self._guard = None  # (K device counter, bound) of the last bounded render
        # the reference's CoreParams::spatial_lr_scale_ is a float (gaussian_model.h): held at
        # f32 precision, so a capture / restore round trip (which stores it as float) is exact
        self.spatial_lr_scale = _f32(spatial_lr_scale)
        # scene extent for the clone / split threshold and the world-size prune; upstream sets
        # spatial_lr_scale to this same value (the nerf++ radius of the training cameras)
        self.cameras_extent = float(spatial_lr_scale if cameras_extent is None else cameras_extent)
        self.k = TrainKernels(dev)
        self.rast = CAbiRasterizer(dev)
        self.gen = torch.Generator(device=dev)
        self.gen.manual_seed(seed)
        self.binning = BinningCapacity(dev)
        self.setup(opt or OptimizationParams())

    @classmethod
    def from_point_cloud(cls, points, colors, max_sh_degree: int, spatial_lr_scale: float,
                         opt: OptimizationParams | None = None, device="cuda", seed: int = 0) -> "GaussianTrainer":
        """Upstream create_from_pcd (the reference has none: its point-cloud branch is commented
        out, src/scene/dataset_readers.cpp:198-219): means = the points, f_dc = RGB2SH(colour),
        f_rest = 0, every scale axis = log(sqrt(max(d, 1e-7))) with d the mean squared distance to
        the 3 nearest other points (gsr_knn_mean_dist2 on the GPU), rotation = (1, 0, 0, 0),
        opacity = inverse_sigmoid(0.1); spatial_lr_scale = the cameras' extent."""
        dev = _device(device)
        pts = torch.as_tensor(np.asarray(points, np.float32), device=dev).reshape(-1, 3).contiguous()
        n = int(pts.shape[0])
        d2 = TrainKernels(dev).knn_mean_dist2(pts)
        scales = torch.log(torch.sqrt(torch.clamp_min(d2, 1e-7)))[:, None].repeat(1, 3)
        rots = torch.zeros((n, 4), dtype=torch.float32, device=dev)
        rots[:, 0] = 1.0
        o = torch.full((n, 1), 0.1, dtype=torch.float32, device=dev)
        opac = torch.log(o / (1 - o))
        rgb = torch.as_tensor(np.asarray(colors, np.float32), device=dev).reshape(-1, 3)
        f_dc = ((rgb - 0.5) / scene_io.SH_C0)[:, None, :]
        f_rest = torch.zeros((n, (max_sh_degree + 1) ** 2 - 1, 3), dtype=torch.float32, device=dev)
        return cls(pts, f_dc, f_rest, opac, scales, rots, max_sh_degree, opt, spatial_lr_scale, dev, seed)

    # ---------------------------------------------------------------- checkpoints / PLY
    def capture(self, path: str) -> None:
        """GaussianModel::capture (src/scene/gaussian_model.cpp:76-131, 228-246): parameters,
        statistics, SH degree, spatial LR scale and every group's Adam state, one file."""
        scene_io.save_checkpoint(path, {
            "active_sh_degree": self.active_sh_degree, "spatial_lr_scale": self.spatial_lr_scale,
            "cameras_extent": self.cameras_extent, "params": self.params, "max_radii2D": self.max_radii2D, "xyz_gradient_accum": self.xyz_gradient_accum,
            "denom": self.denom, "exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq, "steps": self.steps})

    def restore(self, path: str, opt: OptimizationParams | None = None) -> None:
        """GaussianModel::restore (gaussian_model.cpp:248-267): setup(opt), then the captured
        tensors and Adam states replace the fresh ones."""
        st = scene_io.load_checkpoint(path, self.device)
        self.params = {k: v.contiguous() for k, v in st["params"].items()}
        self.spatial_lr_scale = st["spatial_lr_scale"]
        self.cameras_extent = st.get("cameras_extent", self.spatial_lr_scale)
        self.setup(opt or self.opt)
        self.active_sh_degree = st["active_sh_degree"]
        self.max_radii2D, self.xyz_gradient_accum, self.denom = st["max_radii2D"], st["xyz_gradient_accum"], st["denom"]
        for k in self.params:
            if k in st["exp_avg"]:
                self.exp_avg[k] = st["exp_avg"][k].contiguous()
                self.exp_avg_sq[k] = st["exp_avg_sq"][k].contiguous()
                self.steps[k] = st["steps"][k]

    def save_ply(self, path: str) -> None:
        """The raw leaves in the upstream point-cloud PLY layout (scene_io.save_gaussians_ply)."""
        scene_io.save_gaussians_ply(path, **self.params)

    @classmethod
    def from_ply(cls, path: str, max_sh_degree: int, opt: OptimizationParams | None = None,
                 spatial_lr_scale: float = 1.0, device="cuda", seed: int = 0) -> "GaussianTrainer":
        """Upstream load_ply: the leaves of a Gaussian PLY, active SH degree = max_sh_degree."""
        g = scene_io.load_gaussians_ply(path, max_sh_degree)
        tr = cls(g["xyz"], g["f_dc"], g["f_rest"], g["opacity"], g["scaling"], g["rotation"], max_sh_degree, opt,
                 spatial_lr_scale, device, seed)
        tr.active_sh_degree = max_sh_degree
        return tr

    # ---------------------------------------------------------------- GaussianModel surface
    @property
    def num_points(self) -> int:
        return int(self.params["xyz"].shape[0])

    def setup(self, opt: OptimizationParams):
        """GaussianModel::setup (gaussian_model.cpp:316-352)."""
        self.opt = opt
        self.percent_dense = opt.percent_dense
        P = self.num_points
        z = lambda: torch.zeros(P, dtype=torch.float32, device=self.device)
        self.xyz_gradient_accum, self.denom, self.max_radii2D = z(), z(), z()
        self.exp_avg = {k: torch.zeros_like(v) for k, v in self.params.items()}
        self.exp_avg_sq = {k: torch.zeros_like(v) for k, v in self.params.items()}
        self.steps = {k: 0 for k in GROUPS}
        self.lr = {"xyz": opt.position_lr_init * self.spatial_lr_scale, "f_dc": opt.feature_lr,
                   "f_rest": opt.feature_lr / 20.0, "opacity": opt.opacity_lr, "scaling": opt.scaling_lr,
                   "rotation": opt.rotation_lr}
        self.xyz_scheduler = get_expon_lr_func(opt.position_lr_init * self.spatial_lr_scale,
                                               opt.position_lr_final * self.spatial_lr_scale,
                                               lr_delay_steps=0, lr_delay_mult=opt.position_lr_delay_mult,
                                               max_steps=opt.position_lr_max_steps)

    def update_learning_rate(self, iteration: int) -> float:
        lr = self.xyz_scheduler(iteration)
        self.lr["xyz"] = lr
        return lr

    def oneup_SH_degree(self):
        if self.active_sh_degree < self.max_sh_degree:
            self.active_sh_degree += 1

    # ---------------------------------------------------------------- one iteration
    def render(self, cam, bg=(0.0, 0.0, 0.0)):
        s, q, o = self.k.activate(self.params["scaling"], self.params["rotation"], self.params["opacity"])
        p = self.params
        bound = self.binning.bound()
        st = self.rast.forward(cam, p["xyz"], o.reshape(-1), scales=s, rotations=q, sh_dc=p["f_dc"],
                               sh_rest=p["f_rest"] if p["f_rest"].shape[1] else None,
                               sh_degree=self.active_sh_degree, bg=bg, max_rendered=bound)
        # device-side guard of this iteration's statistics / Adam step (see BinningCapacity)
        self._guard = (st.k_device(), bound) if bound > 0 else None
        self.binning.observe(st)
        return st

    def step(self, iteration: int, cam, gt_image: torch.Tensor, bg=(0.0, 0.0, 0.0), densify: bool = True) -> dict:
        """One training iteration in the upstream order (train_utils.cpp:128-145 plus the body
        its stub omits): LR update, SH degree, render, loss, backward, densification statistics,
        densify / prune and opacity reset, then the optimizer step.  As upstream, a group whose
        tensor densification or the opacity reset has just replaced takes no Adam update in
        that iteration (torch Adam skips a fresh parameter, whose .grad is None): a densify
        iteration updates no group, an opacity reset alone skips the opacity group.  Returns
        device tensors (loss stats [loss, l1, ssim], radii); no host synchronisation unless a
        densification is due."""
        opt = self.opt
        self.update_learning_rate(iteration)
        if iteration % 1000 == 0:
            self.oneup_SH_degree()
        st = self.render(cam, bg)
        stats, maps = self.k.loss_forward(st.color, gt_image, opt.lambda_dssim)
        dimg = self.k.loss_backward(st.color, gt_image, opt.lambda_dssim, maps)
        g = self.rast.backward(st, dimg)
        grads = {"xyz": g["means3D"], "f_dc": g["sh_dc"], "opacity": g["opacities"], "scaling": g["scales"],
                 "rotation": g["rotations"]}
        if self.params["f_rest"].shape[1]:
            grads["f_rest"] = g["sh_rest"]
        replaced = set()
        if iteration < opt.densify_until_iter:
            self.k.densify_stats(st.radii, g["means2D"], self.max_radii2D, self.xyz_gradient_accum, self.denom,
                                 guard=self._guard)
            if densify:
                if iteration > opt.densify_from_iter and iteration % opt.densification_interval == 0:
                    size_threshold = 20 if iteration > opt.opacity_reset_interval else None
                    self.densify_and_prune(opt.densify_grad_threshold, 0.005, self.cameras_extent, size_threshold)
                    self.binning.reset()
                    replaced.update(GROUPS)
                if iteration % opt.opacity_reset_interval == 0:
                    self.reset_opacity()
                    self.binning.reset()
                    replaced.add("opacity")
        if iteration < opt.iterations:
            self.optimizer_step({k: v for k, v in grads.items() if k not in replaced})
        return {"stats": stats, "radii": st.radii, "state": st, "image": st.color, "num_points": self.num_points}

    def optimizer_step(self, grads: dict):
        groups = []
        for k in GROUPS:
            if k not in grads:
                continue
            self.steps[k] += 1
            groups.append(dict(param=self.params[k], grad=grads[k].reshape(self.params[k].shape).contiguous(),
                               exp_avg=self.exp_avg[k], exp_avg_sq=self.exp_avg_sq[k], act=ACTS[k],
                               step=self.steps[k], lr=self.lr[k]))
        if groups:
            self.k.adam_step(groups, guard=self._guard)

    # ---------------------------------------------------------------- densification (upstream)
    def _append(self, new: dict):
        """densification_postfix: append rows (zero Adam moments), reset the statistics."""
        for k in GROUPS:
            self.params[k] = torch.cat([self.params[k], new[k].contiguous()], 0).contiguous()
            zeros = torch.zeros_like(new[k])
            self.exp_avg[k] = torch.cat([self.exp_avg[k], zeros], 0).contiguous()
            self.exp_avg_sq[k] = torch.cat([self.exp_avg_sq[k], zeros], 0).contiguous()
        P = self.num_points
        z = lambda: torch.zeros(P, dtype=torch.float32, device=self.device)
        self.xyz_gradient_accum, self.denom, self.max_radii2D = z(), z(), z()

    def prune_points(self, mask: torch.Tensor):
        """Keep the rows where mask is False: one compaction + one multi-tensor gather of the
        parameters, both Adam moments and the three statistics."""
        idx = self.k.compact_index(~mask)
        names = [("p", k) for k in GROUPS] + [("m", k) for k in GROUPS] + [("v", k) for k in GROUPS]
        src = [{"p": self.params, "m": self.exp_avg, "v": self.exp_avg_sq}[a][k] for a, k in names]
        src += [self.xyz_gradient_accum, self.denom, self.max_radii2D]
        out = self.k.gather_rows(src, idx)
        for (a, k), t in zip(names, out):
            {"p": self.params, "m": self.exp_avg, "v": self.exp_avg_sq}[a][k] = t
        self.xyz_gradient_accum, self.denom, self.max_radii2D = out[-3], out[-2], out[-1]

    def _rows(self, mask: torch.Tensor) -> dict:
        idx = self.k.compact_index(mask)
        out = self.k.gather_rows([self.params[k] for k in GROUPS], idx)
        return dict(zip(GROUPS, out))

    def densify_and_clone(self, grads, grad_threshold, scene_extent):
        scaling = torch.exp(self.params["scaling"])
        mask = (grads >= grad_threshold) & (scaling.max(dim=1).values <= self.percent_dense * scene_extent)
        self._append(self._rows(mask))

    def densify_and_split(self, grads, grad_threshold, scene_extent, N=2, samples=None):
        n_init = self.num_points
        padded = torch.zeros(n_init, dtype=torch.float32, device=self.device)
        padded[: grads.shape[0]] = grads
        scaling = torch.exp(self.params["scaling"])
        mask = (padded >= grad_threshold) & (scaling.max(dim=1).values > self.percent_dense * scene_extent)
        sel = self._rows(mask)
        stds = torch.exp(sel["scaling"]).repeat(N, 1)
        if samples is None:
            samples = torch.normal(torch.zeros_like(stds), stds, generator=self.gen)
        rots = build_rotation(sel["rotation"]).repeat(N, 1, 1)
        new = {"xyz": torch.bmm(rots, samples.unsqueeze(-1)).squeeze(-1) + sel["xyz"].repeat(N, 1),
               "scaling": torch.log(torch.exp(sel["scaling"]).repeat(N, 1) / (0.8 * N)),
               "rotation": sel["rotation"].repeat(N, 1), "f_dc": sel["f_dc"].repeat(N, 1, 1),
               "f_rest": sel["f_rest"].repeat(N, 1, 1), "opacity": sel["opacity"].repeat(N, 1)}
        self._append(new)
        prune = torch.cat([mask, torch.zeros(N * int(sel["xyz"].shape[0]), dtype=torch.bool, device=self.device)])
        self.prune_points(prune)

    def densify_and_prune(self, max_grad, min_opacity, extent, max_screen_size, split_samples=None):
        grads = self.xyz_gradient_accum / self.denom
        grads[grads.isnan()] = 0.0
        self.densify_and_clone(grads, max_grad, extent)
        self.densify_and_split(grads, max_grad, extent, samples=split_samples)
        prune = (torch.sigmoid(self.params["opacity"]) < min_opacity).squeeze(1)
        if max_screen_size:
            big_vs = self.max_radii2D > max_screen_size
            big_ws = torch.exp(self.params["scaling"]).max(dim=1).values > 0.1 * extent
            prune = prune | big_vs | big_ws
        self.prune_points(prune)

    def reset_opacity(self):
        o = torch.sigmoid(self.params["opacity"])
        o = torch.minimum(o, torch.full_like(o, 0.01))
        self.params["opacity"] = torch.log(o / (1 - o)).contiguous()  # inverse_sigmoid
        self.exp_avg["opacity"].zero_()
        self.exp_avg_sq["opacity"].zero_()
