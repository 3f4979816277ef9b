"""Deterministic synthetic Gaussian clouds for the parity tests and bench.

Portable PRNG: SplitMix64, one independent counter-based stream per attribute, uniform
``u = (x >> 40) * 2**-24``, normals by Box-Muller in float64 rounded to f32.  CPU oracle
and GPU consume the *same* f32 arrays (generated once, on the host).

Returned arrays are the rasterizer's *activated* inputs (the caller of render() applies
``exp`` / ``sigmoid`` / ``normalize`` as GaussianModel's getters do,
src/scene/gaussian_model.cpp:270-298) plus the raw parameters for autograd tests.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

from .graphics import RasterCamera

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)

# attribute stream ids
_S_MEANS, _S_SCALE, _S_ROT, _S_OPAC, _S_DC, _S_REST, _S_DPIX = range(7)


def splitmix64(seed: int, stream: int, n: int) -> np.ndarray:
    """n outputs of SplitMix64 seeded with mix(seed, stream); counter-based."""
    base = np.uint64((seed * 0x100000001B3 + stream * 0xD6E8FEB86659FD93) & 0xFFFFFFFFFFFFFFFF)
    with np.errstate(over="ignore"):
        z = base + (np.arange(1, n + 1, dtype=np.uint64) * _GOLDEN)
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    return z


def uniform(seed: int, stream: int, n: int) -> np.ndarray:
    """float64 in [0, 1) with 24 random bits."""
    return (splitmix64(seed, stream, n) >> np.uint64(40)).astype(np.float64) * (2.0 ** -24)


def normal(seed: int, stream: int, n: int) -> np.ndarray:
    """float64 standard normals (Box-Muller, cos branch)."""
    u = uniform(seed, stream, 2 * n)
    u1, u2 = 1.0 - u[0::2], u[1::2]
    return np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * math.pi * u2)


@dataclass
class SyntheticScene:
    P: int
    max_sh_degree: int
    means3D: np.ndarray    # (P,3) f32
    scales: np.ndarray     # (P,3) f32, activated (exp)
    rotations: np.ndarray  # (P,4) f32, normalised (w,x,y,z)
    opacities: np.ndarray  # (P,1) f32, activated (sigmoid)
    sh_dc: np.ndarray      # (P,1,3) f32
    sh_rest: np.ndarray    # (P,M-1,3) f32, M=(max_sh_degree+1)^2
    raw_scales: np.ndarray
    raw_rotations: np.ndarray
    raw_opacities: np.ndarray


def make_scene(cam: RasterCamera, P: int, max_sh_degree: int = 3, seed: int = 0,
               opacity_sigma: float = 1.5) -> SyntheticScene:
    """SURVEY §8d distributions:
    z ~ U[2,12]; x = (2u-1) 1.1 z tanfovx; y = (2u-1) 1.1 z tanfovy;
    log s_k = log(3 px * z / f_x) + 0.5 n;  rotation raw ~ N(0,1)^4 (normalised);
    opacity raw = clamp(N(0, 1.5), -6, 4.5) (sigmoid <= 0.989 < 0.99: alpha clamp never hit);
    SH dc ~ N(0, 0.3), rest ~ N(0, 0.05)."""
    u = uniform(seed, _S_MEANS, 3 * P).reshape(P, 3)
    z = 2.0 + 10.0 * u[:, 2]
    x = (2.0 * u[:, 0] - 1.0) * 1.1 * z * cam.tanfovx
    y = (2.0 * u[:, 1] - 1.0) * 1.1 * z * cam.tanfovy
    means = np.stack([x, y, z], axis=1).astype(np.float32)
    fx = cam.width / (2.0 * cam.tanfovx)
    n_s = normal(seed, _S_SCALE, 3 * P).reshape(P, 3)
    raw_scales = (np.log(3.0 * z / fx)[:, None] + 0.5 * n_s).astype(np.float32)
    raw_rot = normal(seed, _S_ROT, 4 * P).reshape(P, 4).astype(np.float32)
    raw_op = np.clip(opacity_sigma * normal(seed, _S_OPAC, P), -6.0, 4.5).astype(np.float32)[:, None]
    M = (max_sh_degree + 1) ** 2
    dc = (0.3 * normal(seed, _S_DC, 3 * P)).astype(np.float32).reshape(P, 1, 3)
    rest = (0.05 * normal(seed, _S_REST, 3 * (M - 1) * P)).astype(np.float32).reshape(P, M - 1, 3)
    # activations in float64, then rounded (identical bytes for CPU and GPU)
    scales = np.exp(raw_scales.astype(np.float64)).astype(np.float32)
    r64 = raw_rot.astype(np.float64)
    rot = (r64 / np.maximum(np.linalg.norm(r64, axis=1, keepdims=True), 1e-12)).astype(np.float32)
    opac = (1.0 / (1.0 + np.exp(-raw_op.astype(np.float64)))).astype(np.float32)
    return SyntheticScene(P=P, max_sh_degree=max_sh_degree, means3D=means, scales=scales,
                          rotations=rot, opacities=opac, sh_dc=dc, sh_rest=rest,
                          raw_scales=raw_scales, raw_rotations=raw_rot, raw_opacities=raw_op)


def make_dL_dpix(cam: RasterCamera, seed: int = 1) -> np.ndarray:
    """Upstream image gradient U[-1,1], shape (3,H,W), seed+1 stream."""
    n = 3 * cam.width * cam.height
    return (2.0 * uniform(seed, _S_DPIX, n) - 1.0).astype(np.float32).reshape(3, cam.height, cam.width)
