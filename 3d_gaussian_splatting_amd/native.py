"""Loader for the native libraries + a ctypes binding of the C ABI (include/gsr/gsr.h).

Product path, no fallback: if lib/libgsr_hip.so or the libtorch extension is missing this
module raises -- it never substitutes a CPU implementation.

The ctypes structures and argtypes below are the stub a Python (or any FFI) caller binds: the
parity tests drive the HIP kernels through them directly (gsr_forward / gsr_backward /
gsr_backward_blend / gsr_backward_preprocess / the multi-GPU gsr_shard_* / gsr_band_* split /
gsr_view), with device memory owned by torch tensors.
"""
from __future__ import annotations

import ctypes
import importlib.machinery
import importlib.util
import os

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(PKG, "lib")
# GSR_HIP_LIB: an experiment build (lib/variants/<name>/libgsr_hip.so) instead of the shipped one
HIP_LIB = os.environ.get("GSR_HIP_LIB") or os.path.join(LIB_DIR, "libgsr_hip.so")

ABI_VERSION = 4
GSR_FLAG_DEBUG = 1
GSR_FLAG_ROW_SPANS = 2  # gsr.h: gsr_shard_forward row_hist = 3 x grid_y (instances, rect start rows, end rows)
GSR_ERR_OVERFLOW = -4
GSR_GRAD2D_STRIDE = 12
GSR_MAX_BATCH = 64
GSR_MAX_VIEWS = 8
GSR_SPLAT_BYTES = 64
GSR_SPLAT_GRAD_BYTES = 48
MAX_BANDS = 16
VIEW_SORTED_GID, VIEW_SORTED_TILE, VIEW_RANGES, VIEW_FINAL_T, VIEW_N_CONTRIB, VIEW_DEPTH_KEY, \
    VIEW_TILES_TOUCHED, VIEW_RECORDS, VIEW_COUNTS, VIEW_TERM, VIEW_CK_LIVE = range(1, 12)
TERM_STRIDE = 32  # GSR_TERM_STRIDE: words per tile of VIEW_TERM
CK_DIV = 48       # a tile of n instances opens at most n // CK_DIV B1 chunks (gsr.h, VIEW_CK_LIVE)


def ck_slot(fixed: bool, start: int, tile: int, chunk: int) -> int:
    """B1 checkpoint slot of a tile's chunk >= 1 (gsr.h GSR_VIEW_CK_LIVE)."""
    return tile * (TERM_STRIDE - 1) + chunk - 1 if fixed else start // CK_DIV + tile + chunk - 1
EXPORTS = ["gsr_abi_version", "gsr_last_error", "gsr_forward", "gsr_read_num_rendered", "gsr_forward_batch",
           "gsr_forward_views", "gsr_backward_views", "gsr_backward", "gsr_backward_blend", "gsr_backward_preprocess", "gsr_shard_forward",
           "gsr_band_forward", "gsr_band_backward", "gsr_shard_backward", "gsr_exchange_block_bytes",
           "gsr_shard_state_bytes", "gsr_view", "gsr_geom_bytes", "gsr_binning_bytes",
           "gsr_image_bytes", "gsr_scratch_bytes", "gsr_ck_pool_slots", "gsr_profile_enable", "gsr_profile_read",
           "gsr_stage_name", "gsr_band_publish", "gsr_gather_finish"]
# include/gsr/gsr_train.h (training-step kernels)
TRAIN_EXPORTS = ["gsr_activate", "gsr_loss_scratch_bytes", "gsr_loss_forward", "gsr_loss_backward", "gsr_adam_step",
                 "gsr_adam_step_guarded", "gsr_densify_stats", "gsr_densify_stats_guarded", "gsr_compact_scratch_bytes", "gsr_compact_index", "gsr_gather_rows",
                 "gsr_knn_scratch_bytes", "gsr_knn_mean_dist2"]
COMM_EXPORTS = ["gsr_comm_unique_id", "gsr_comm_init", "gsr_comm_destroy", "gsr_comm_size", "gsr_comm_all_to_all",
                "gsr_comm_all_gather", "gsr_comm_all_reduce_i64"]  # include/gsr/gsr_comm.h
COMM_ID_BYTES = 128
ACT_NONE, ACT_EXP, ACT_SIGMOID, ACT_NORMALIZE4 = range(4)
ADAM_MAX_GROUPS = 8
GATHER_MAX = 24
STAGES = ["preprocess", "depth_sort", "scan", "duplicate", "tile_sort", "finalize", "blend_fwd", "blend_bwd",
          "preprocess_bwd", "gather_grad2d", "misc", "exchange"]


class Camera(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32),
                ("tanfovx", ctypes.c_float), ("tanfovy", ctypes.c_float),
                ("viewmatrix", ctypes.c_float * 16), ("projmatrix", ctypes.c_float * 16),
                ("campos", ctypes.c_float * 3)]


class Gaussians(ctypes.Structure):
    _fields_ = [("P", ctypes.c_int32), ("sh_degree", ctypes.c_int32), ("sh_rest_coeffs", ctypes.c_int32),
                ("scale_modifier", ctypes.c_float)] + [
        (n, ctypes.c_void_p) for n in ("means3D", "sh_dc", "sh_rest", "colors_precomp", "opacities",
                                       "scales", "rotations", "cov3D_precomp")]


class Settings(ctypes.Structure):
    _fields_ = [("bg", ctypes.c_float * 3), ("tile_y0", ctypes.c_int32), ("tile_y1", ctypes.c_int32),
                ("flags", ctypes.c_uint32), ("max_rendered", ctypes.c_int32)]


class Grads(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in (
        "dL_dmeans2D", "dL_dconic", "dL_dopacity", "dL_dcolors", "dL_dmeans3D", "dL_dsh_dc",
        "dL_dsh_rest", "dL_dscales", "dL_drotations", "dL_dcov3D")]


class Buffers(ctypes.Structure):
    _fields_ = [("geom", ctypes.c_void_p), ("binning", ctypes.c_void_p), ("image", ctypes.c_void_p),
                ("num_rendered", ctypes.c_int32), ("capacity", ctypes.c_int32), ("n_local", ctypes.c_int32),
                ("layout", ctypes.c_uint32)]


class AdamGroup(ctypes.Structure):
    _fields_ = [("param", ctypes.c_void_p), ("grad", ctypes.c_void_p), ("exp_avg", ctypes.c_void_p),
                ("exp_avg_sq", ctypes.c_void_p), ("n", ctypes.c_int64), ("act", ctypes.c_int32),
                ("step", ctypes.c_int32), ("lr", ctypes.c_float)]


class RowCopy(ctypes.Structure):
    _fields_ = [("src", ctypes.c_void_p), ("dst", ctypes.c_void_p), ("width", ctypes.c_int32)]


ALLOC_FN = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)

_hip = None
_ext = None


def hip_library_path() -> str:
    return HIP_LIB


def load_hip() -> ctypes.CDLL:
    """dlopen libgsr_hip.so (after torch, so the process has ONE HIP runtime)."""
    global _hip
    if _hip is None:
        import torch  # noqa: F401  (loads torch's libamdhip64.so.7 first)
        if not os.path.exists(HIP_LIB):
            raise RuntimeError(f"{HIP_LIB} missing: run __graft_entry__.build() (no CPU fallback)")
        L = ctypes.CDLL(HIP_LIB, mode=ctypes.RTLD_GLOBAL)
        vp, i32 = ctypes.c_void_p, ctypes.c_int32
        L.gsr_abi_version.restype = ctypes.c_int
        L.gsr_last_error.restype = ctypes.c_char_p
        L.gsr_forward.restype = ctypes.c_int
        L.gsr_forward.argtypes = [ctypes.POINTER(Camera), ctypes.POINTER(Gaussians), ctypes.POINTER(Settings),
                                  vp, vp, ALLOC_FN, ALLOC_FN, ALLOC_FN, vp, ctypes.POINTER(Buffers), vp]
        L.gsr_read_num_rendered.restype = ctypes.c_int
        L.gsr_read_num_rendered.argtypes = [ctypes.POINTER(Camera), ctypes.POINTER(Buffers), ctypes.POINTER(i32), vp]
        L.gsr_forward_batch.restype = ctypes.c_int
        L.gsr_forward_batch.argtypes = [i32, ctypes.POINTER(Camera), ctypes.POINTER(Gaussians),
                                        ctypes.POINTER(Settings), ctypes.POINTER(vp), ctypes.POINTER(vp), ALLOC_FN,
                                        ALLOC_FN, ALLOC_FN, vp, ctypes.POINTER(Buffers), vp]
        L.gsr_forward_views.restype = ctypes.c_int
        L.gsr_forward_views.argtypes = [i32, ctypes.POINTER(Camera), ctypes.POINTER(Gaussians),
                                        ctypes.POINTER(Settings), vp, vp, ALLOC_FN, ALLOC_FN, ALLOC_FN, vp,
                                        ctypes.POINTER(Buffers), vp]
        L.gsr_backward_views.restype = ctypes.c_int
        L.gsr_backward_views.argtypes = [i32, ctypes.POINTER(Camera), ctypes.POINTER(Gaussians),
                                         ctypes.POINTER(Settings), ctypes.POINTER(Buffers), vp, ALLOC_FN, vp,
                                         ctypes.POINTER(Grads), vp]
        L.gsr_backward.restype = ctypes.c_int
        L.gsr_backward.argtypes = [ctypes.POINTER(Camera), ctypes.POINTER(Gaussians), ctypes.POINTER(Settings),
                                   ctypes.POINTER(Buffers), vp, ALLOC_FN, vp, ctypes.POINTER(Grads), vp]
        L.gsr_backward_blend.restype = ctypes.c_int
        L.gsr_backward_blend.argtypes = [ctypes.POINTER(Camera), ctypes.POINTER(Gaussians),
                                         ctypes.POINTER(Settings), ctypes.POINTER(Buffers), vp, ALLOC_FN, vp,
                                         vp, vp]
        L.gsr_backward_preprocess.restype = ctypes.c_int
        L.gsr_backward_preprocess.argtypes = [ctypes.POINTER(Camera), ctypes.POINTER(Gaussians),
                                              ctypes.POINTER(Settings), ctypes.POINTER(Buffers), vp,
                                              ctypes.POINTER(Grads), vp]
        # multi-GPU split: shard F1 + pack, band F2..F6, band B1, shard sum + B2
        pi32 = ctypes.POINTER(i32)
        L.gsr_exchange_block_bytes.restype = ctypes.c_size_t
        L.gsr_exchange_block_bytes.argtypes = [i32]
        L.gsr_shard_state_bytes.restype = ctypes.c_size_t
        L.gsr_shard_state_bytes.argtypes = [i32, i32, i32]
        L.gsr_shard_forward.restype = ctypes.c_int
        L.gsr_shard_forward.argtypes = [ctypes.POINTER(Camera), ctypes.POINTER(Gaussians), ctypes.POINTER(Settings),
                                        i32, pi32, i32, vp, vp, vp, vp, vp]
        L.gsr_band_forward.restype = ctypes.c_int
        L.gsr_band_forward.argtypes = [ctypes.POINTER(Camera), ctypes.POINTER(Settings), i32, i32, vp, vp,
                                       ALLOC_FN, ALLOC_FN, ALLOC_FN, vp, ctypes.POINTER(Buffers), vp]
        L.gsr_band_backward.restype = ctypes.c_int
        L.gsr_band_backward.argtypes = [ctypes.POINTER(Camera), ctypes.POINTER(Settings), i32, i32,
                                        ctypes.POINTER(Buffers), vp, ALLOC_FN, vp, vp, vp]
        L.gsr_shard_backward.restype = ctypes.c_int
        L.gsr_shard_backward.argtypes = [ctypes.POINTER(Camera), ctypes.POINTER(Gaussians), ctypes.POINTER(Settings),
                                         i32, pi32, i32, vp, vp, ctypes.POINTER(Grads), vp]
        L.gsr_view.restype = vp
        L.gsr_view.argtypes = [ctypes.POINTER(Camera), i32, ctypes.POINTER(Buffers), ctypes.c_int]
        for n in ("gsr_geom_bytes", "gsr_scratch_bytes"):
            getattr(L, n).restype = ctypes.c_size_t
            getattr(L, n).argtypes = [i32]
        for n in ("gsr_binning_bytes", "gsr_ck_pool_slots"):
            getattr(L, n).restype = ctypes.c_size_t
            getattr(L, n).argtypes = [i32, i32, i32]
        L.gsr_profile_enable.restype = ctypes.c_int
        L.gsr_profile_enable.argtypes = [ctypes.c_uint32]
        L.gsr_profile_read.restype = ctypes.c_int
        L.gsr_profile_read.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint32)]
        L.gsr_stage_name.restype = ctypes.c_char_p
        L.gsr_stage_name.argtypes = [ctypes.c_int]
        L.gsr_image_bytes.restype = ctypes.c_size_t
        L.gsr_image_bytes.argtypes = [i32, i32]
        # gsr_train.h
        f32 = ctypes.c_float
        L.gsr_activate.restype = ctypes.c_int
        L.gsr_activate.argtypes = [vp, vp, vp, i32, vp, vp, vp, vp]
        L.gsr_loss_scratch_bytes.restype = ctypes.c_size_t
        L.gsr_loss_scratch_bytes.argtypes = [i32, i32, i32]
        L.gsr_loss_forward.restype = ctypes.c_int
        L.gsr_loss_forward.argtypes = [vp, vp, i32, i32, i32, f32, vp, vp, vp]
        L.gsr_loss_backward.restype = ctypes.c_int
        L.gsr_loss_backward.argtypes = [vp, vp, i32, i32, i32, f32, vp, vp, vp]
        L.gsr_adam_step.restype = ctypes.c_int
        L.gsr_adam_step.argtypes = [ctypes.POINTER(AdamGroup), i32, f32, f32, f32, vp]
        L.gsr_adam_step_guarded.restype = ctypes.c_int
        L.gsr_adam_step_guarded.argtypes = [ctypes.POINTER(AdamGroup), i32, f32, f32, f32, vp, ctypes.c_uint32, vp]
        L.gsr_densify_stats.restype = ctypes.c_int
        L.gsr_densify_stats.argtypes = [vp, vp, i32, vp, vp, vp, vp]
        L.gsr_densify_stats_guarded.restype = ctypes.c_int
        L.gsr_densify_stats_guarded.argtypes = [vp, vp, i32, vp, vp, vp, vp, ctypes.c_uint32, vp]
        L.gsr_compact_scratch_bytes.restype = ctypes.c_size_t
        L.gsr_compact_scratch_bytes.argtypes = [i32]
        L.gsr_compact_index.restype = ctypes.c_int
        L.gsr_compact_index.argtypes = [vp, i32, vp, vp, vp, vp]
        L.gsr_gather_rows.restype = ctypes.c_int
        L.gsr_gather_rows.argtypes = [ctypes.POINTER(RowCopy), i32, vp, i32, vp]
        L.gsr_knn_scratch_bytes.restype = ctypes.c_size_t
        L.gsr_knn_scratch_bytes.argtypes = [i32]
        L.gsr_knn_mean_dist2.restype = ctypes.c_int
        L.gsr_knn_mean_dist2.argtypes = [vp, i32, vp, vp, vp]
        _hip = L
    return _hip


def load_torch_ext():
    """Import lib/_gsr_torch*.so (the libtorch RasterizeGaussians layer)."""
    global _ext
    if _ext is None:
        import torch  # noqa: F401
        load_hip()
        from . import _build
        path = os.path.join(LIB_DIR, _build.torch_ext_name())
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run __graft_entry__.build() (no CPU fallback)")
        loader = importlib.machinery.ExtensionFileLoader("_gsr_torch", path)
        spec = importlib.util.spec_from_file_location("_gsr_torch", path, loader=loader)
        mod = importlib.util.module_from_spec(spec)
        loader.exec_module(mod)
        _ext = mod
    return _ext


def camera_struct(cam) -> Camera:
    c = Camera()
    c.width, c.height = int(cam.width), int(cam.height)
    c.tanfovx, c.tanfovy = float(cam.tanfovx), float(cam.tanfovy)
    c.viewmatrix[:] = [float(v) for v in cam.viewmatrix]
    c.projmatrix[:] = [float(v) for v in cam.projmatrix]
    c.campos[:] = [float(v) for v in cam.campos]
    return c


def profile_enable(mask: int = (1 << len(STAGES)) - 1) -> None:
    load_hip().gsr_profile_enable(mask)


def profile_read() -> dict:
    """{stage: (total_ms, launches)} accumulated since profile_enable (syncs the events)."""
    L = load_hip()
    ms = (ctypes.c_double * len(STAGES))()
    cnt = (ctypes.c_uint32 * len(STAGES))()
    L.gsr_profile_read(ms, cnt)
    return {STAGES[i]: (float(ms[i]), int(cnt[i])) for i in range(len(STAGES))}


def last_error() -> str:
    return load_hip().gsr_last_error().decode()
