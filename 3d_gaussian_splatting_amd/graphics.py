"""Camera / view math the rasterizer consumes (host side, float64 like the reference).

Restates the reference's graphics utilities and Camera matrix construction:
  - ``focal2fov``              src/utils/graphics_utils.cpp:4-7
  - ``get_world2view``         src/utils/graphics_utils.cpp:10-29   (Rt = [R^T | t])
  - ``get_world2view_2``       src/utils/graphics_utils.cpp:32-43
  - ``get_projection_matrix``  src/utils/graphics_utils.cpp:46-72
  - ``Camera`` matrices        src/scene/camera.cpp:66-71 (world_view_transform =
    world2view_2^T, full_proj = world_view @ proj^T, camera_center = inv(world_view)[3,:3];
    znear 0.01 / zfar 100 from camera.cpp:44-45)

``RasterCamera`` is the POD the rasterizer boundary consumes: f32 matrices
in the column-major layout a kernel reads as ``m[0..15]`` (i.e. the row-vector-convention
4x4 tensors of camera.cpp flattened row-major), plus tan(fov/2) and the image size.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np


def focal2fov(focal: float, pixels: float) -> float:
    """graphics_utils.cpp:4-7."""
    return 2.0 * math.atan(pixels / (2.0 * focal))


def fov2focal(fov: float, pixels: float) -> float:
    return pixels / (2.0 * math.tan(fov / 2.0))


def get_world2view(R: np.ndarray, t: np.ndarray) -> np.ndarray:
    """graphics_utils.cpp:10-29: upper-left = R^T, last column = t."""
    Rt = np.zeros((4, 4), dtype=np.float64)
    Rt[:3, :3] = np.asarray(R, dtype=np.float64).T
    Rt[:3, 3] = np.asarray(t, dtype=np.float64)
    Rt[3, 3] = 1.0
    return Rt


def get_world2view_2(R, t, translate=(0.0, 0.0, 0.0), scale: float = 1.0) -> np.ndarray:
    """graphics_utils.cpp:32-43: re-centre / re-scale the camera centre."""
    Rt = get_world2view(R, t)
    C2W = np.linalg.inv(Rt)
    cam_center = (C2W[:3, 3] + np.asarray(translate, dtype=np.float64)) * scale
    C2W[:3, 3] = cam_center
    return np.linalg.inv(C2W)


def get_projection_matrix(znear: float, zfar: float, fovX: float, fovY: float) -> np.ndarray:
    """graphics_utils.cpp:46-72 (z_sign = 1)."""
    tan_y = math.tan(fovY / 2.0)
    tan_x = math.tan(fovX / 2.0)
    top = tan_y * znear
    bottom = -top
    right = tan_x * znear
    left = -right
    P = np.zeros((4, 4), dtype=np.float64)
    z_sign = 1.0
    P[0, 0] = 2.0 * znear / (right - left)
    P[1, 1] = 2.0 * znear / (top - bottom)
    P[0, 2] = (right + left) / (right - left)
    P[1, 2] = (top + bottom) / (top - bottom)
    P[3, 2] = z_sign
    P[2, 2] = z_sign * zfar / (zfar - znear)
    P[2, 3] = -(zfar * znear) / (zfar - znear)
    return P


@dataclass
class RasterCamera:
    """POD view description handed to the rasterizer (f32, column-major matrices)."""

    width: int
    height: int
    tanfovx: float
    tanfovy: float
    viewmatrix: np.ndarray = field(repr=False)  # (16,) f32: world_view_transform (row-major flat)
    projmatrix: np.ndarray = field(repr=False)  # (16,) f32: full_proj_transform (row-major flat)
    campos: np.ndarray = field(repr=False)      # (3,) f32
    znear: float = 0.01
    zfar: float = 100.0

    @property
    def grid(self) -> tuple[int, int]:
        return ((self.width + 15) // 16, (self.height + 15) // 16)


def make_camera(R, T, FoVx: float, FoVy: float, width: int, height: int,
                trans=(0.0, 0.0, 0.0), scale: float = 1.0,
                znear: float = 0.01, zfar: float = 100.0) -> RasterCamera:
    """Build the rasterizer camera exactly as camera.cpp:66-71 builds its tensors
    (float64), then cast to f32 at the boundary."""
    world_view = get_world2view_2(R, T, trans, scale).T
    proj = get_projection_matrix(znear, zfar, FoVx, FoVy).T
    full_proj = world_view @ proj
    camera_center = np.linalg.inv(world_view)[3, :3]
    return RasterCamera(
        width=int(width), height=int(height),
        tanfovx=float(np.float32(math.tan(FoVx * 0.5))),
        tanfovy=float(np.float32(math.tan(FoVy * 0.5))),
        viewmatrix=np.ascontiguousarray(world_view, dtype=np.float32).reshape(16),
        projmatrix=np.ascontiguousarray(full_proj, dtype=np.float32).reshape(16),
        campos=np.ascontiguousarray(camera_center, dtype=np.float32),
        znear=znear, zfar=zfar)


def synthetic_camera(width: int, height: int, fovx_deg: float = 60.0) -> RasterCamera:
    """SURVEY §8d benchmark camera: R = I, T = 0 (looking down +z), FoVx = 60 deg,
    FoVy = 2 atan(tan(FoVx/2) H / W)."""
    fovx = math.radians(fovx_deg)
    fovy = 2.0 * math.atan(math.tan(fovx / 2.0) * height / width)
    return make_camera(np.eye(3), np.zeros(3), fovx, fovy, width, height)
