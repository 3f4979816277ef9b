"""Python mirror of the rasterizer surface.

Two entry points, both ending in the same HIP kernels:

* ``CAbiRasterizer`` -- drives the C ABI (include/gsr/gsr.h) through ctypes with torch-owned
  device memory: what a ctypes / cgo / JNI binding of libgsr_hip.so looks like.  The GPU parity
  tests and bench.py use it so every call crosses the C boundary.
* ``render()`` / ``rasterize_gaussians()`` -- the libtorch RasterizeGaussians autograd Function
  (lib/_gsr_torch*.so), i.e. the C++ render() surface (csrc/torch/gsr_render.h) the
  reference's training loop would call at src/utils/train_utils.cpp:137-144.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np
import torch

from . import native
from .graphics import RasterCamera

INT32_MAX = 2**31 - 1


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _f32(t, shape=None, device=None):
    if t is None:
        return None
    t = torch.as_tensor(t, dtype=torch.float32, device=device)
    if shape is not None:
        t = t.reshape(shape)
    return t.contiguous()


class _Allocator:
    """Allocation callbacks for the C ABI: uint8 tensors kept alive by the owner.  With `reuse`
    (a list kept by the caller across calls), the i-th request of a call gets the i-th tensor
    of the previous call when it is large enough -- a step loop then allocates nothing (the
    previous step's buffers are dead by the time the next step's kernels run: one stream)."""

    def __init__(self, device, reuse: list | None = None):
        self.device = device
        self.tensors = []
        self.reuse = reuse
        self.cb = native.ALLOC_FN(self._alloc)

    def _alloc(self, _ctx, nbytes):
        n = max(int(nbytes), 16)
        i = len(self.tensors)
        if self.reuse is not None and i < len(self.reuse) and self.reuse[i].numel() >= n:
            t = self.reuse[i]
        else:
            t = torch.empty(n, dtype=torch.uint8, device=self.device)
            if self.reuse is not None:
                if i < len(self.reuse):
                    self.reuse[i] = t
                else:
                    self.reuse.append(t)
        self.tensors.append(t)
        return t.data_ptr()


@dataclass
class ForwardState:
    cam: RasterCamera
    inputs: dict
    settings: native.Settings
    gauss: native.Gaussians
    buffers: native.Buffers
    color: torch.Tensor
    radii: torch.Tensor
    allocs: list = field(default_factory=list)

    @property
    def num_rendered(self) -> int:
        """K.  Under a binning bound (max_rendered > 0) K stays on the device until asked for:
        the first access reads it back (synchronising the stream) and raises on an overflow."""
        if self.buffers.num_rendered < 0:
            L = native.load_hip()
            c = native.camera_struct(self.cam)
            k = ctypes.c_int32(0)
            rc = L.gsr_read_num_rendered(ctypes.byref(c), ctypes.byref(self.buffers), ctypes.byref(k),
                                         ctypes.c_void_p(torch.cuda.current_stream(self.color.device).cuda_stream))
            if rc == native.GSR_ERR_OVERFLOW:
                raise OverflowError(native.last_error())
            if rc != 0:
                raise RuntimeError(f"gsr_read_num_rendered failed ({rc}): {native.last_error()}")
            self.buffers.num_rendered = k.value
        return int(self.buffers.num_rendered)

    def _owner(self, ptr: int):
        for a in self.allocs:
            for t in a.tensors:
                base = t.data_ptr()
                if base <= ptr < base + t.numel():
                    return t, ptr - base
        raise KeyError("pointer not inside a forward buffer")

    def k_device(self) -> torch.Tensor:
        """K as a 1-element int32 device tensor aliasing the scan's counter (no copy, no sync)."""
        L = native.load_hip()
        c = native.camera_struct(self.cam)
        p = L.gsr_view(ctypes.byref(c), self.gauss.P, ctypes.byref(self.buffers), native.VIEW_COUNTS)
        if not p:
            raise RuntimeError("gsr_view(COUNTS) returned NULL")
        t, off = self._owner(p)
        return t[off:off + 4].view(torch.int32)

    def view(self, what: int, dtype: torch.dtype, count: int) -> torch.Tensor:
        """Copy of an internal array (gsr_view) as a torch tensor."""
        L = native.load_hip()
        c = native.camera_struct(self.cam)
        p = L.gsr_view(ctypes.byref(c), self.gauss.P, ctypes.byref(self.buffers), what)
        if not p or count == 0:
            return torch.empty(0, dtype=dtype, device=self.color.device)
        t, off = self._owner(p)
        nbytes = count * torch.empty(0, dtype=dtype).element_size()
        return t[off:off + nbytes].view(dtype).clone()


@dataclass
class ViewsState:
    """gsr_forward_views' outputs, kept for gsr_backward_views (one set of buffers for all views)."""
    cams: list
    cstructs: object          # the gsr_camera array handed to the library
    inputs: dict
    settings: native.Settings
    gauss: native.Gaussians
    buffers: native.Buffers
    color: torch.Tensor       # V x 3 x H x W
    radii: torch.Tensor       # V x P
    allocs: list

    @property
    def num_rendered(self) -> int:
        """K over all views.  Under a binning bound (max_rendered > 0) it is read back on first
        access through gsr_read_num_rendered with the pass's tall camera (the views stacked as
        bands of ceil(H / 16) tile rows), raising on an overflow."""
        if self.buffers.num_rendered < 0:
            L = native.load_hip()
            tall = native.Camera()
            ctypes.memmove(ctypes.byref(tall), ctypes.byref(self.cstructs[0]), ctypes.sizeof(tall))
            tall.height = len(self.cams) * ((self.cams[0].height + 15) // 16) * 16
            k = ctypes.c_int32(0)
            rc = L.gsr_read_num_rendered(ctypes.byref(tall), ctypes.byref(self.buffers), ctypes.byref(k),
                                         ctypes.c_void_p(torch.cuda.current_stream(self.color.device).cuda_stream))
            if rc == native.GSR_ERR_OVERFLOW:
                raise OverflowError(native.last_error())
            if rc != 0:
                raise RuntimeError(f"gsr_read_num_rendered failed ({rc}): {native.last_error()}")
            self.buffers.num_rendered = k.value
        return int(self.buffers.num_rendered)

    def tall_camera(self):
        """The pass's camera struct: the views stacked as bands of ceil(H / 16) tile rows."""
        tall = native.Camera()
        ctypes.memmove(ctypes.byref(tall), ctypes.byref(self.cstructs[0]), ctypes.sizeof(tall))
        tall.height = len(self.cams) * ((self.cams[0].height + 15) // 16) * 16
        return tall

    def view(self, what: int, dtype: torch.dtype, count: int) -> torch.Tensor:
        """Copy of an internal array of the pass (gsr_view over the tall grid and the V * P
        (view, Gaussian) entries e = v * P + g): sorted tiles are tall-grid tile ids, sorted gids
        are entry ids."""
        L = native.load_hip()
        tall = self.tall_camera()
        p = L.gsr_view(ctypes.byref(tall), len(self.cams) * self.gauss.P, ctypes.byref(self.buffers), what)
        if not p or count == 0:
            return torch.empty(0, dtype=dtype, device=self.color.device)
        nbytes = count * torch.empty(0, dtype=dtype).element_size()
        for a in self.allocs:
            for t in a.tensors:
                base = t.data_ptr()
                if base <= p < base + t.numel():
                    return t[p - base:p - base + nbytes].view(dtype).clone()
        raise KeyError("pointer not inside a views buffer")


class CAbiRasterizer:
    """Thin ctypes front-end of gsr_forward / gsr_backward*."""

    def __init__(self, device="cuda"):
        self.device = torch.device(device)
        self.L = native.load_hip()
        self._cams = {}  # camera contents -> gsr_camera struct

    @staticmethod
    def _cam_key(cam):
        """Everything camera_struct reads, by value: an in-place edit of a camera's matrices or
        size gives a new key, never a stale struct (a stale width / height would size the
        kernels' writes differently from the colour tensor made from the new camera)."""
        return (int(cam.width), int(cam.height), float(cam.tanfovx), float(cam.tanfovy),
                np.asarray(cam.viewmatrix, np.float32).tobytes(), np.asarray(cam.projmatrix, np.float32).tobytes(),
                np.asarray(cam.campos, np.float32).tobytes())

    def _cam(self, cam):
        key = self._cam_key(cam)
        c = self._cams.get(key)
        if c is not None:
            return c
        c = native.camera_struct(cam)
        if len(self._cams) > 256:
            self._cams.clear()
        self._cams[key] = c
        return c

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _check(self, rc, what):
        if rc != 0:
            raise RuntimeError(f"{what} failed ({rc}): {native.last_error()}")

    def _prepare(self, means3D, opacities, scales, rotations, sh_dc, sh_rest, sh_degree, colors_precomp,
                 cov3D_precomp, scale_modifier, bg, tile_rows, max_rendered, debug):
        dev = self.device
        means3D = _f32(means3D, device=dev)
        P = int(means3D.shape[0])
        inputs = dict(means3D=means3D.reshape(P, 3), opacities=_f32(opacities, (P,), dev),
                      scales=_f32(scales, (P, 3), dev) if scales is not None else None,
                      rotations=_f32(rotations, (P, 4), dev) if rotations is not None else None,
                      sh_dc=_f32(sh_dc, (P, 1, 3), dev) if sh_dc is not None else None,
                      sh_rest=_f32(sh_rest, device=dev) if sh_rest is not None else None,
                      colors_precomp=_f32(colors_precomp, (P, 3), dev) if colors_precomp is not None else None,
                      cov3D_precomp=_f32(cov3D_precomp, (P, 6), dev) if cov3D_precomp is not None else None)
        if inputs["sh_rest"] is not None:
            inputs["sh_rest"] = inputs["sh_rest"].reshape(P, -1, 3).contiguous()
            if inputs["sh_rest"].shape[1] == 0:
                inputs["sh_rest"] = None
        g = native.Gaussians()
        g.P, g.sh_degree, g.scale_modifier = P, int(sh_degree), float(scale_modifier)
        g.sh_rest_coeffs = 0 if inputs["sh_rest"] is None else int(inputs["sh_rest"].shape[1])
        for k in ("means3D", "sh_dc", "sh_rest", "colors_precomp", "opacities", "scales", "rotations",
                  "cov3D_precomp"):
            setattr(g, k, None if inputs[k] is None else inputs[k].data_ptr())
        s = native.Settings()
        s.bg[:] = [float(v) for v in bg]
        s.tile_y0, s.tile_y1 = (0, INT32_MAX) if tile_rows is None else (int(tile_rows[0]), int(tile_rows[1]))
        s.flags = native.GSR_FLAG_DEBUG if debug else 0
        s.max_rendered = int(max_rendered)
        return inputs, g, s

    def forward(self, cam: RasterCamera, means3D, opacities, scales=None, rotations=None, sh_dc=None,
                sh_rest=None, sh_degree=0, colors_precomp=None, cov3D_precomp=None, scale_modifier=1.0,
                bg=(0.0, 0.0, 0.0), tile_rows=None, max_rendered=0, debug=False) -> ForwardState:
        """gsr_forward.  max_rendered > 0 sizes the binning for that many instances and skips the
        host read of K (see ForwardState.num_rendered)."""
        dev = self.device
        inputs, g, s = self._prepare(means3D, opacities, scales, rotations, sh_dc, sh_rest, sh_degree,
                                     colors_precomp, cov3D_precomp, scale_modifier, bg, tile_rows, max_rendered,
                                     debug)
        P = g.P
        color = torch.empty((3, cam.height, cam.width), dtype=torch.float32, device=dev)
        radii = torch.empty((P,), dtype=torch.int32, device=dev)
        ag, ab, ai = _Allocator(dev), _Allocator(dev), _Allocator(dev)
        bufs = native.Buffers()
        c = self._cam(cam)
        rc = self.L.gsr_forward(ctypes.byref(c), ctypes.byref(g), ctypes.byref(s), _ptr(color),
                                _ptr(radii) if P else None, ag.cb, ab.cb, ai.cb, None, ctypes.byref(bufs),
                                self._stream())
        self._check(rc, "gsr_forward")
        return ForwardState(cam=cam, inputs=inputs, settings=s, gauss=g, buffers=bufs, color=color,
                            radii=radii, allocs=[ag, ab, ai])

    def forward_batch(self, cams, means3D, opacities, scales=None, rotations=None, sh_dc=None, sh_rest=None,
                      sh_degree=0, colors_precomp=None, cov3D_precomp=None, scale_modifier=1.0,
                      bg=(0.0, 0.0, 0.0), max_rendered=0, debug=False) -> list:
        """gsr_forward_batch: one ForwardState per camera (full images), one host wait in total
        (none with max_rendered > 0)."""
        dev = self.device
        inputs, g, s = self._prepare(means3D, opacities, scales, rotations, sh_dc, sh_rest, sh_degree,
                                     colors_precomp, cov3D_precomp, scale_modifier, bg, None, max_rendered, debug)
        V, P = len(cams), g.P
        colors = [torch.empty((3, c.height, c.width), dtype=torch.float32, device=dev) for c in cams]
        radii = [torch.empty((P,), dtype=torch.int32, device=dev) for _ in cams]
        ag, ab, ai = _Allocator(dev), _Allocator(dev), _Allocator(dev)
        bufs = (native.Buffers * V)()
        cs = (native.Camera * V)(*[native.camera_struct(c) for c in cams])
        col_p = (ctypes.c_void_p * V)(*[t.data_ptr() for t in colors])
        rad_p = (ctypes.c_void_p * V)(*[t.data_ptr() for t in radii])
        rc = self.L.gsr_forward_batch(V, cs, ctypes.byref(g), ctypes.byref(s), col_p, rad_p if P else None, ag.cb,
                                      ab.cb, ai.cb, None, bufs, self._stream())
        self._check(rc, "gsr_forward_batch")
        out = []
        for v, cam in enumerate(cams):
            b = native.Buffers()
            ctypes.memmove(ctypes.byref(b), ctypes.byref(bufs[v]), ctypes.sizeof(b))
            out.append(ForwardState(cam=cam, inputs=inputs, settings=s, gauss=g, buffers=b, color=colors[v],
                                    radii=radii[v], allocs=[ag, ab, ai]))
        return out

    def forward_views(self, cams, means3D, opacities, scales=None, rotations=None, sh_dc=None, sh_rest=None,
                      sh_degree=0, colors_precomp=None, cov3D_precomp=None, scale_modifier=1.0,
                      bg=(0.0, 0.0, 0.0), max_rendered=0, debug=False) -> "ViewsState":
        """gsr_forward_views: V same-size cameras in one pass (one launch per stage).  color is
        V x 3 x H x W, radii V x P; bit-identical to V forward() calls."""
        dev = self.device
        inputs, g, s = self._prepare(means3D, opacities, scales, rotations, sh_dc, sh_rest, sh_degree,
                                     colors_precomp, cov3D_precomp, scale_modifier, bg, None, max_rendered, debug)
        V, P = len(cams), g.P
        H, W = cams[0].height, cams[0].width
        color = torch.empty((V, 3, H, W), dtype=torch.float32, device=dev)
        radii = torch.empty((V, P), dtype=torch.int32, device=dev)
        ag, ab, ai = _Allocator(dev), _Allocator(dev), _Allocator(dev)
        bufs = native.Buffers()
        cs = (native.Camera * V)(*[self._cam(c) for c in cams])
        rc = self.L.gsr_forward_views(V, cs, ctypes.byref(g), ctypes.byref(s), _ptr(color),
                                      _ptr(radii) if P else None, ag.cb, ab.cb, ai.cb, None, ctypes.byref(bufs),
                                      self._stream())
        self._check(rc, "gsr_forward_views")
        return ViewsState(cams=list(cams), cstructs=cs, inputs=inputs, settings=s, gauss=g, buffers=bufs,
                          color=color, radii=radii, allocs=[ag, ab, ai])

    def backward_views(self, st: "ViewsState", dL_dpix) -> dict:
        """gsr_backward_views: means2D / conic gradients per view (V x P x 3), leaf gradients
        summed over the views in view order."""
        V = len(st.cams)
        dpix = _f32(dL_dpix, (V, 3, st.cams[0].height, st.cams[0].width), self.device)
        out, gg = self._grad_tensors(st)
        P = st.gauss.P
        for k, name in (("means2D", "dL_dmeans2D"), ("conic", "dL_dconic")):
            out[k] = torch.empty((V, P, 3), dtype=torch.float32, device=self.device)
            setattr(gg, name, out[k].data_ptr())
        scratch = _Allocator(self.device)
        rc = self.L.gsr_backward_views(V, st.cstructs, ctypes.byref(st.gauss), ctypes.byref(st.settings),
                                       ctypes.byref(st.buffers), _ptr(dpix), scratch.cb, None, ctypes.byref(gg),
                                       self._stream())
        self._check(rc, "gsr_backward_views")
        return out

    def _grad_tensors(self, st: ForwardState, P: int | None = None):
        P = st.gauss.P if P is None else P
        dev = self.device
        e = lambda *shape: torch.empty(shape, dtype=torch.float32, device=dev)
        out = dict(means2D=e(P, 3), conic=e(P, 3), opacities=e(P, 1), means3D=e(P, 3))
        inp = st.inputs
        if inp["colors_precomp"] is not None:
            out["colors"] = e(P, 3)
        else:
            out["sh_dc"] = e(P, 1, 3)
            if inp["sh_rest"] is not None:
                out["sh_rest"] = inp["sh_rest"].new_empty((P,) + tuple(inp["sh_rest"].shape[1:]))
        if inp["cov3D_precomp"] is not None:
            out["cov3D"] = e(P, 6)
        else:
            out["scales"], out["rotations"] = e(P, 3), e(P, 4)
        gg = native.Grads()
        names = dict(means2D="dL_dmeans2D", conic="dL_dconic", opacities="dL_dopacity", colors="dL_dcolors",
                     means3D="dL_dmeans3D", sh_dc="dL_dsh_dc", sh_rest="dL_dsh_rest", scales="dL_dscales",
                     rotations="dL_drotations", cov3D="dL_dcov3D")
        for k, v in out.items():
            setattr(gg, names[k], v.data_ptr())
        return out, gg

    def backward(self, st: ForwardState, dL_dpix) -> dict:
        dpix = _f32(dL_dpix, (3, st.cam.height, st.cam.width), self.device)
        out, gg = self._grad_tensors(st)
        scratch = _Allocator(self.device)
        c = self._cam(st.cam)
        rc = self.L.gsr_backward(ctypes.byref(c), ctypes.byref(st.gauss), ctypes.byref(st.settings),
                                 ctypes.byref(st.buffers), _ptr(dpix), scratch.cb, None, ctypes.byref(gg),
                                 self._stream())
        self._check(rc, "gsr_backward")
        return out

    def backward_blend(self, st: ForwardState, dL_dpix, out: torch.Tensor | None = None) -> torch.Tensor:
        """B1 + per-Gaussian sum -> grad2d (P x 12).  `out`: optional contiguous (>= P) x 12
        tensor to write into."""
        dpix = _f32(dL_dpix, (3, st.cam.height, st.cam.width), self.device)
        if out is None:
            grad2d = torch.empty((st.gauss.P, native.GSR_GRAD2D_STRIDE), dtype=torch.float32, device=self.device)
        else:
            if not (out.is_contiguous() and out.dtype == torch.float32 and out.shape[0] >= st.gauss.P
                    and out.shape[1] == native.GSR_GRAD2D_STRIDE):
                raise ValueError("backward_blend: out must be a contiguous f32 (>= P) x 12 tensor")
            grad2d = out
        scratch = _Allocator(self.device)
        c = self._cam(st.cam)
        rc = self.L.gsr_backward_blend(ctypes.byref(c), ctypes.byref(st.gauss), ctypes.byref(st.settings),
                                       ctypes.byref(st.buffers), _ptr(dpix), scratch.cb, None, _ptr(grad2d),
                                       self._stream())
        self._check(rc, "gsr_backward_blend")
        return grad2d

    def backward_preprocess(self, st: ForwardState, grad2d: torch.Tensor) -> dict:
        out, gg = self._grad_tensors(st)
        grad2d = grad2d.contiguous()
        c = self._cam(st.cam)
        rc = self.L.gsr_backward_preprocess(ctypes.byref(c), ctypes.byref(st.gauss), ctypes.byref(st.settings),
                                            ctypes.byref(st.buffers), _ptr(grad2d), ctypes.byref(gg),
                                            self._stream())
        self._check(rc, "gsr_backward_preprocess")
        return out


# ------------------------------------------------------------------------------------------
# multi-GPU split (gsr_shard_* / gsr_band_*): the compute of one rank
# ------------------------------------------------------------------------------------------
@dataclass
class ShardState:
    """gsr_shard_forward's outputs a rank keeps until gsr_shard_backward."""
    cam: RasterCamera
    inputs: dict
    settings: native.Settings
    gauss: native.Gaussians
    band_rows: list
    pair_cap: int
    send: torch.Tensor        # nbands exchange blocks (uint8)
    state: torch.Tensor       # gsr_shard_state_bytes (uint8)
    radii: torch.Tensor

    @property
    def counts(self) -> torch.Tensor:
        """Splats packed per band (device u32 headers; > pair_cap = overflow)."""
        nb = len(self.band_rows) - 1
        blk = self.send.numel() // nb
        return self.send.view(nb, blk).view(torch.int32)[:, 0]  # strided view of the headers


class ShardRasterizer(CAbiRasterizer):
    """The per-rank calls of the multi-GPU path; the caller moves the exchange blocks."""

    def block_bytes(self, pair_cap: int) -> int:
        return int(self.L.gsr_exchange_block_bytes(int(pair_cap)))

    def shard_forward(self, cam: RasterCamera, band_rows, pair_cap: int, means3D, opacities, scales=None,
                      rotations=None, sh_dc=None, sh_rest=None, sh_degree=0, colors_precomp=None,
                      cov3D_precomp=None, scale_modifier=1.0, row_hist: torch.Tensor | None = None,
                      debug=False, reuse: dict | None = None, row_spans: bool = False) -> ShardState:
        """`reuse` (a dict the caller keeps across steps): the send / state / radii buffers and the
        prepared input structs of the previous call with the same sizes are used again.
        row_hist (zeroed by the caller) += the instances per tile row; with row_spans it holds
        3 x grid_y u32: that, then the rect start rows and end rows (GSR_FLAG_ROW_SPANS)."""
        dev = self.device
        srcs = (means3D, opacities, scales, rotations, sh_dc, sh_rest, colors_precomp, cov3D_precomp)
        key = None
        if all(t is None or (torch.is_tensor(t) and t.is_contiguous() and t.dtype == torch.float32
                             and t.device == dev) for t in srcs):
            key = tuple(None if t is None else (t.data_ptr(), tuple(t.shape)) for t in srcs) + \
                (int(sh_degree), float(scale_modifier), bool(debug))
        if reuse is not None and key is not None and reuse.get("key") == key:
            inputs, g, s = reuse["prep"]
        else:
            inputs, g, s = self._prepare(means3D, opacities, scales, rotations, sh_dc, sh_rest, sh_degree,
                                         colors_precomp, cov3D_precomp, scale_modifier, (0.0, 0.0, 0.0), None, 0,
                                         debug)
            if reuse is not None:
                reuse["key"], reuse["prep"] = key, (inputs, g, s)
        nb = len(band_rows) - 1
        rows = (ctypes.c_int32 * (nb + 1))(*[int(r) for r in band_rows])
        nsend = nb * self.block_bytes(pair_cap)
        nstate = int(self.L.gsr_shard_state_bytes(g.P, nb, int(pair_cap)))
        if reuse is not None and reuse.get("sizes") == (nsend, nstate, g.P):
            send, state, radii = reuse["bufs"]
        else:
            send = torch.empty(nsend, dtype=torch.uint8, device=dev)
            state = torch.empty(nstate, dtype=torch.uint8, device=dev)
            radii = torch.empty((g.P,), dtype=torch.int32, device=dev)
            if reuse is not None:
                reuse["sizes"], reuse["bufs"] = (nsend, nstate, g.P), (send, state, radii)
        c = self._cam(cam)
        s.flags = (native.GSR_FLAG_DEBUG if debug else 0) | (native.GSR_FLAG_ROW_SPANS if row_spans else 0)
        if row_spans and (row_hist is None or row_hist.numel() < 3 * ((cam.height + 15) // 16)):
            raise ValueError("row_spans needs a row_hist of 3 x grid_y words")
        rc = self.L.gsr_shard_forward(ctypes.byref(c), ctypes.byref(g), ctypes.byref(s), nb, rows, int(pair_cap),
                                      _ptr(send), _ptr(radii) if g.P else None, _ptr(state), _ptr(row_hist),
                                      self._stream())
        self._check(rc, "gsr_shard_forward")
        return ShardState(cam=cam, inputs=inputs, settings=s, gauss=g, band_rows=list(band_rows),
                          pair_cap=int(pair_cap), send=send, state=state, radii=radii)

    def band_forward(self, cam: RasterCamera, tile_rows, nsrc: int, pair_cap: int, recv: torch.Tensor,
                     max_rendered: int, out_color: torch.Tensor | None = None, bg=(0.0, 0.0, 0.0),
                     debug=False, reuse: dict | None = None) -> ForwardState:
        """F2..F6 over the splats received from nsrc shards; only the band's pixels of
        out_color are written.  `reuse`: the caller's dict of buffers kept across steps."""
        dev = self.device
        s = native.Settings()
        s.bg[:] = [float(v) for v in bg]
        s.tile_y0, s.tile_y1 = int(tile_rows[0]), int(tile_rows[1])
        s.flags = native.GSR_FLAG_DEBUG if debug else 0
        s.max_rendered = int(max_rendered)
        if out_color is not None:
            color = out_color
        elif reuse is not None and "color" in reuse and tuple(reuse["color"].shape) == (3, cam.height, cam.width):
            color = reuse["color"]  # the band's pixels are rewritten; the rest stay as they were
        else:
            color = torch.zeros((3, cam.height, cam.width), dtype=torch.float32, device=dev)
            if reuse is not None:
                reuse["color"] = color
        r = (lambda k: reuse.setdefault(k, [])) if reuse is not None else (lambda k: None)
        ag, ab, ai = _Allocator(dev, r("geom")), _Allocator(dev, r("bin")), _Allocator(dev, r("img"))
        bufs = native.Buffers()
        c = self._cam(cam)
        rc = self.L.gsr_band_forward(ctypes.byref(c), ctypes.byref(s), int(nsrc), int(pair_cap), _ptr(recv),
                                     _ptr(color), ag.cb, ab.cb, ai.cb, None, ctypes.byref(bufs), self._stream())
        self._check(rc, "gsr_band_forward")
        g = native.Gaussians()
        g.P = int(nsrc) * int(pair_cap)
        return ForwardState(cam=cam, inputs={"recv": recv}, settings=s, gauss=g, buffers=bufs, color=color,
                            radii=torch.empty(0, dtype=torch.int32, device=dev), allocs=[ag, ab, ai])

    def band_backward(self, st: ForwardState, nsrc: int, pair_cap: int, dL_dpix, reuse: dict | None = None) -> torch.Tensor:
        """B1 + per-splat 2D gradients in the received slot layout: (nsrc * pair_cap, 12) f32."""
        dpix = _f32(dL_dpix, (3, st.cam.height, st.cam.width), self.device)
        shape = (int(nsrc) * int(pair_cap), native.GSR_GRAD2D_STRIDE)
        if reuse is not None and "g2" in reuse and tuple(reuse["g2"].shape) == shape:
            out = reuse["g2"]
        else:
            out = torch.empty(shape, dtype=torch.float32, device=self.device)
            if reuse is not None:
                reuse["g2"] = out
        scratch = _Allocator(self.device, reuse.setdefault("scratch", []) if reuse is not None else None)
        c = self._cam(st.cam)
        rc = self.L.gsr_band_backward(ctypes.byref(c), ctypes.byref(st.settings), int(nsrc), int(pair_cap),
                                      ctypes.byref(st.buffers), _ptr(dpix), scratch.cb, None, _ptr(out),
                                      self._stream())
        self._check(rc, "gsr_band_backward")
        return out

    def shard_backward(self, sh: ShardState, grad_recv: torch.Tensor, reuse: dict | None = None) -> dict:
        """Sum of the bands' 2D gradients per Gaussian (band order), then B2 on the shard."""
        st = ForwardState(cam=sh.cam, inputs=sh.inputs, settings=sh.settings, gauss=sh.gauss,
                          buffers=native.Buffers(), color=sh.radii, radii=sh.radii)
        if reuse is not None and reuse.get("grads_P") == sh.gauss.P:
            out, gg = reuse["grads"]
        else:
            out, gg = self._grad_tensors(st)
            if reuse is not None:
                reuse["grads_P"], reuse["grads"] = sh.gauss.P, (out, gg)
        nb = len(sh.band_rows) - 1
        rows = (ctypes.c_int32 * (nb + 1))(*[int(r) for r in sh.band_rows])
        c = self._cam(sh.cam)
        rc = self.L.gsr_shard_backward(ctypes.byref(c), ctypes.byref(sh.gauss), ctypes.byref(sh.settings), nb, rows,
                                       sh.pair_cap, _ptr(sh.state), _ptr(grad_recv.contiguous()), ctypes.byref(gg),
                                       self._stream())
        self._check(rc, "gsr_shard_backward")
        return out


# ------------------------------------------------------------------------------------------
# autograd surface (libtorch extension)
# ------------------------------------------------------------------------------------------
def ext_camera(cam: RasterCamera):
    ext = native.load_torch_ext()
    return ext.RasterCamera(cam.width, cam.height, float(cam.tanfovx), float(cam.tanfovy),
                            [float(v) for v in cam.viewmatrix], [float(v) for v in cam.projmatrix],
                            [float(v) for v in cam.campos])


def rasterize_gaussians(cam: RasterCamera, means3D, means2D, opacities, sh_dc=None, sh_rest=None,
                        colors_precomp=None, scales=None, rotations=None, cov3D_precomp=None,
                        sh_degree=0, scale_modifier=1.0, bg=(0.0, 0.0, 0.0), tile_rows=None, debug=False,
                        max_rendered=0):
    """RasterizeGaussians.apply: returns (color (3,H,W), radii (P,) int32); differentiable in
    every tensor input (means2D receives the screen-space gradient)."""
    ext = native.load_torch_ext()
    y0, y1 = (0, INT32_MAX) if tile_rows is None else tile_rows
    rs = ext.RasterSettings([float(v) for v in bg], float(scale_modifier), int(sh_degree), int(y0), int(y1),
                            bool(debug), int(max_rendered))
    return ext.rasterize_gaussians(ext_camera(cam), rs, means3D, means2D, sh_dc, sh_rest, colors_precomp,
                                   opacities, scales, rotations, cov3D_precomp)


@dataclass
class PipelineParams:
    """Mirror of src/arguments/params.h:93-106."""
    convert_SHs_python: bool = False
    compute_cov3D_python: bool = False
    debug: bool = False


def render(viewpoint_camera: RasterCamera, pc, pipe: PipelineParams, bg_color, scaling_modifier=1.0,
           override_color=None) -> dict:
    """render(): same contract as the C++ gsr::render template (csrc/torch/gsr_render.h) for a
    model exposing the reference GaussianModel getters (see model.GaussianModel)."""
    from .general import eval_sh
    xyz = pc.get_xyz
    screenspace = torch.zeros_like(xyz, requires_grad=True)
    bg = [float(v) for v in torch.as_tensor(bg_color).flatten().tolist()]
    scales = rotations = cov3D = sh_dc = sh_rest = colors = None
    if pipe.compute_cov3D_python:
        cov3D = pc.get_covariance(scaling_modifier)
    else:
        scales, rotations = pc.get_scaling, pc.get_rotation
    if override_color is not None:
        colors = override_color
    elif pipe.convert_SHs_python:
        campos = torch.as_tensor(viewpoint_camera.campos, device=xyz.device)
        dirs = xyz - campos
        dirs = dirs / dirs.norm(dim=1, keepdim=True)
        colors = torch.clamp_min(eval_sh(pc.active_sh_degree, pc.get_features, dirs) + 0.5, 0.0)
    else:
        sh_dc, sh_rest = pc.features_dc, pc.features_rest
    color, radii = rasterize_gaussians(viewpoint_camera, xyz, screenspace, pc.get_opacity, sh_dc=sh_dc,
                                       sh_rest=sh_rest, colors_precomp=colors, scales=scales,
                                       rotations=rotations, cov3D_precomp=cov3D,
                                       sh_degree=0 if colors is not None else pc.active_sh_degree,
                                       scale_modifier=scaling_modifier, bg=bg, debug=pipe.debug)
    return dict(render=color, viewspace_points=screenspace, visibility_filter=radii > 0, radii=radii)
