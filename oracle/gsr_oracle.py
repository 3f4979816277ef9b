"""ctypes front-end of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module,
and only as the checker / reported CPU baseline (see gsr_oracle.h for what it restates).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libgsr_oracle.so")
_lib = None


class _Cam(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int), ("height", ctypes.c_int),
                ("tanfovx", ctypes.c_float), ("tanfovy", ctypes.c_float),
                ("viewmatrix", ctypes.c_float * 16), ("projmatrix", ctypes.c_float * 16),
                ("campos", ctypes.c_float * 3)]


def build(force: bool = False) -> str:
    if force or not os.path.exists(_LIB_PATH):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB_PATH)
        fp = ctypes.POINTER(ctypes.c_float)
        ip = ctypes.POINTER(ctypes.c_int)
        up = ctypes.POINTER(ctypes.c_uint32)
        vp = ctypes.c_void_p
        L.gsro_forward.restype = ctypes.c_int
        L.gsro_forward.argtypes = [ctypes.POINTER(_Cam), ctypes.c_int, ctypes.c_int, ctypes.c_int, fp,
                                   fp, fp, fp, fp, fp, fp, ctypes.c_float, fp, fp, ctypes.c_int,
                                   ctypes.c_int, fp, ip, ctypes.POINTER(vp)]
        L.gsro_backward.restype = ctypes.c_int
        L.gsro_backward.argtypes = [vp, fp] + [fp] * 10
        L.gsro_free.argtypes = [vp]
        L.gsro_num_rendered.argtypes = [vp]
        L.gsro_num_rendered.restype = ctypes.c_int
        L.gsro_get_sorted.argtypes = [vp, up, up, up]
        L.gsro_get_ranges.argtypes = [vp, up]
        L.gsro_get_pixel_state.argtypes = [vp, fp, up]
        L.gsro_get_preprocess.argtypes = [vp, fp, fp, fp, fp, up]
        L.gsro_forward_pairs.argtypes = [vp]
        L.gsro_get_examined.argtypes = [vp, up]
        L.gsro_forward_pairs.restype = ctypes.c_uint64
        L.gsro_blend_work.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64)]
        L.gsro_build_rotation.argtypes = [fp, fp]
        L.gsro_covariance.argtypes = [fp, ctypes.c_float, fp, fp]
        _lib = L
    return _lib


def _f(a):
    if a is None:
        return None
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _u(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))


def _c32(a):
    return None if a is None else np.ascontiguousarray(a, dtype=np.float32)


def cam_struct(cam) -> _Cam:
    c = _Cam()
    c.width, c.height = cam.width, cam.height
    c.tanfovx, c.tanfovy = cam.tanfovx, cam.tanfovy
    c.viewmatrix[:] = [float(v) for v in cam.viewmatrix]
    c.projmatrix[:] = [float(v) for v in cam.projmatrix]
    c.campos[:] = [float(v) for v in cam.campos]
    return c


@dataclass
class OracleForward:
    color: np.ndarray
    radii: np.ndarray
    num_rendered: int
    state: "OracleState"


class OracleState:
    """Owns the C state and the input arrays it borrows."""

    def __init__(self, ptr, keep, cam, P, M_rest, has_colors, has_cov):
        self.ptr = ptr
        self._keep = keep
        self.cam = cam
        self.P = P
        self.M_rest = M_rest
        self.has_colors = has_colors
        self.has_cov = has_cov

    def __del__(self):
        if getattr(self, "ptr", None):
            lib().gsro_free(self.ptr)
            self.ptr = None

    @property
    def num_rendered(self) -> int:
        return lib().gsro_num_rendered(self.ptr)

    def sorted(self):
        K = self.num_rendered
        t = np.zeros(K, np.uint32); d = np.zeros(K, np.uint32); g = np.zeros(K, np.uint32)
        lib().gsro_get_sorted(self.ptr, _u(t), _u(d), _u(g))
        return t, d, g

    def ranges(self):
        gx, gy = self.cam.grid
        r = np.zeros(gx * gy * 2, np.uint32)
        lib().gsro_get_ranges(self.ptr, _u(r))
        return r.reshape(gx * gy, 2)

    def pixel_state(self):
        H, W = self.cam.height, self.cam.width
        T = np.zeros(H * W, np.float32); n = np.zeros(H * W, np.uint32)
        lib().gsro_get_pixel_state(self.ptr, _f(T), _u(n))
        return T.reshape(H, W), n.reshape(H, W)

    def preprocess(self):
        P = self.P
        xy = np.zeros((P, 2), np.float32); depth = np.zeros(P, np.float32)
        co = np.zeros((P, 4), np.float32); rgb = np.zeros((P, 3), np.float32)
        tt = np.zeros(P, np.uint32)
        lib().gsro_get_preprocess(self.ptr, _f(xy), _f(depth), _f(co), _f(rgb), _u(tt))
        return dict(xy=xy, depth=depth, conic_o=co, rgb=rgb, tiles_touched=tt)

    def examined(self):
        H, W = self.cam.height, self.cam.width
        e = np.zeros(H * W, np.uint32)
        lib().gsro_get_examined(self.ptr, _u(e))
        return e.reshape(H, W)

    def forward_pairs(self) -> int:
        return int(lib().gsro_forward_pairs(self.ptr))

    def blend_work(self) -> dict:
        """The blend kernels' culled work (gsro_blend_work): lower bounds of F6's wave visits and
        B1's stripe evaluations (all / with a contributing pixel) and visited entries."""
        w = (ctypes.c_uint64 * 4)()
        lib().gsro_blend_work(self.ptr, w)
        return dict(f6_wave_visits=int(w[0]), b1_stripe_evals=int(w[1]), b1_contrib_evals=int(w[2]),
                    b1_records=int(w[3]))

    def backward(self, dL_dpix: np.ndarray) -> dict:
        P, Mr = self.P, self.M_rest
        dpix = np.ascontiguousarray(dL_dpix, dtype=np.float32)
        out = dict(
            means2D=np.zeros((P, 3), np.float32), conic=np.zeros((P, 3), np.float32),
            opacities=np.zeros((P, 1), np.float32), colors=np.zeros((P, 3), np.float32),
            means3D=np.zeros((P, 3), np.float32), sh_dc=np.zeros((P, 1, 3), np.float32),
            sh_rest=np.zeros((P, max(Mr, 0), 3), np.float32), scales=np.zeros((P, 3), np.float32),
            rotations=np.zeros((P, 4), np.float32), cov3D=np.zeros((P, 6), np.float32))
        rc = lib().gsro_backward(self.ptr, _f(dpix), _f(out["means2D"]), _f(out["conic"]),
                                 _f(out["opacities"]), _f(out["colors"]), _f(out["means3D"]),
                                 _f(out["sh_dc"]), _f(out["sh_rest"]) if Mr > 0 else None,
                                 _f(out["scales"]), _f(out["rotations"]), _f(out["cov3D"]))
        if rc != 0:
            raise RuntimeError(f"gsro_backward failed: {rc}")
        return out


def forward(cam, means3D, opacities, scales=None, rotations=None, sh_dc=None, sh_rest=None,
            sh_degree: int = 0, colors_precomp=None, cov3D_precomp=None, scale_modifier=1.0,
            bg=(0.0, 0.0, 0.0), tile_rows=None) -> OracleForward:
    """Oracle forward on host arrays; mirrors gsr_forward's argument meaning."""
    P = int(np.asarray(means3D).shape[0])
    means3D = _c32(means3D).reshape(P, 3)
    opacities = _c32(opacities).reshape(P)
    scales = _c32(scales); rotations = _c32(rotations)
    sh_dc = _c32(sh_dc); sh_rest = _c32(sh_rest)
    colors_precomp = _c32(colors_precomp); cov3D_precomp = _c32(cov3D_precomp)
    M_rest = 0 if sh_rest is None else int(sh_rest.reshape(P, -1).shape[1] // 3)
    bg = np.ascontiguousarray(bg, dtype=np.float32)
    H, W = cam.height, cam.width
    color = np.zeros((3, H, W), np.float32)
    radii = np.zeros(P, np.int32)
    y0, y1 = (0, 1 << 30) if tile_rows is None else tile_rows
    st = ctypes.c_void_p()
    c = cam_struct(cam)
    rc = lib().gsro_forward(ctypes.byref(c), P, int(sh_degree), M_rest, _f(bg), _f(means3D), _f(sh_dc),
                            _f(sh_rest), _f(colors_precomp), _f(opacities), _f(scales),
                            float(scale_modifier), _f(rotations), _f(cov3D_precomp), int(y0), int(y1),
                            _f(color), radii.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
                            ctypes.byref(st))
    if rc < 0:
        raise RuntimeError(f"gsro_forward failed: {rc}")
    keep = (means3D, opacities, scales, rotations, sh_dc, sh_rest, colors_precomp, cov3D_precomp, bg)
    state = OracleState(st, keep, cam, P, M_rest, colors_precomp is not None, cov3D_precomp is not None)
    return OracleForward(color=color, radii=radii, num_rendered=rc, state=state)


def build_rotation(q) -> np.ndarray:
    q = _c32(q).reshape(4)
    R = np.zeros(9, np.float32)
    lib().gsro_build_rotation(_f(q), _f(R))
    return R.reshape(3, 3)


def covariance(s, mod, q) -> np.ndarray:
    s = _c32(s).reshape(3); q = _c32(q).reshape(4)
    c = np.zeros(6, np.float32)
    lib().gsro_covariance(_f(s), float(mod), _f(q), _f(c))
    return c
