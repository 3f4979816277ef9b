"""Minimal GaussianModel exposing the reference's getter surface (what render() consumes).

Mirrors src/scene/gaussian_model.h:9-40,85-90 / gaussian_model.cpp:37-62,270-313: raw leaves
(xyz, features_dc, features_rest, scaling, rotation, opacity), activations exp / sigmoid /
normalize, get_covariance via build_covariance_from_scaling_rotation, active_sh_degree with
oneup_SH_degree.  Optimiser / densification / checkpointing are out of scope.
"""
from __future__ import annotations

import torch

from .general import build_covariance_from_scaling_rotation
from .scene import SyntheticScene


class GaussianModel:
    def __init__(self, sh_degree: int):
        self.max_sh_degree = sh_degree
        self.active_sh_degree = 0
        self._xyz = self._features_dc = self._features_rest = None
        self._scaling = self._rotation = self._opacity = None

    @classmethod
    def from_scene(cls, s: SyntheticScene, device="cuda", active_sh_degree=None) -> "GaussianModel":
        m = cls(s.max_sh_degree)
        m.active_sh_degree = s.max_sh_degree if active_sh_degree is None else active_sh_degree
        leaf = lambda a: torch.tensor(a, dtype=torch.float32, device=device).requires_grad_(True)
        m._xyz = leaf(s.means3D)
        m._features_dc = leaf(s.sh_dc)
        m._features_rest = leaf(s.sh_rest)
        m._scaling = leaf(s.raw_scales)
        m._rotation = leaf(s.raw_rotations)
        m._opacity = leaf(s.raw_opacities)
        return m

    # getters (gaussian_model.cpp:270-304)
    @property
    def get_xyz(self):
        return self._xyz

    @property
    def get_scaling(self):
        return torch.exp(self._scaling)

    @property
    def get_rotation(self):
        return torch.nn.functional.normalize(self._rotation, p=2, dim=1)

    @property
    def get_opacity(self):
        return torch.sigmoid(self._opacity)

    @property
    def get_features(self):
        return torch.cat([self._features_dc, self._features_rest], dim=1)

    @property
    def features_dc(self):
        return self._features_dc

    @property
    def features_rest(self):
        return self._features_rest

    def get_covariance(self, scaling_modifier=1.0):
        return build_covariance_from_scaling_rotation(self.get_scaling, scaling_modifier, self._rotation)

    def oneup_SH_degree(self):
        if self.active_sh_degree < self.max_sh_degree:
            self.active_sh_degree += 1

    def parameters(self):
        return [self._xyz, self._features_dc, self._features_rest, self._scaling, self._rotation, self._opacity]
