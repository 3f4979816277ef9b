#!/usr/bin/env python3
"""Per-tile list lengths of the training-loop workload (bench.py --mode loop defaults): the
initial model (train_loop.synthetic_scene -> GaussianTrainer.from_point_cloud) rendered from a
few of its cameras.  Sizes the per-tile depth sort's forms for real-scene densities."""
import importlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "3d_gaussian_splatting_amd"
L = importlib.import_module(f"{PKG}.train_loop")
T = importlib.import_module(f"{PKG}.trainer")
native = importlib.import_module(f"{PKG}.native")

dev = torch.device("cuda", 0)
scene = L.synthetic_scene(4_000_000, 1_000_000, 16, 1280, 832, seed=0, device=dev, texture=1.0)
tr = T.GaussianTrainer.from_point_cloud(scene.points, scene.colors, 3, spatial_lr_scale=scene.extent, device=dev)
for v in (0, 5, 10):
    st = tr.render(scene.cams[v])
    gx, gy = scene.cams[v].grid
    rng = st.view(native.VIEW_RANGES, torch.int32, 2 * gx * gy).cpu().numpy().reshape(-1, 2)
    n = rng[:, 1] - rng[:, 0]
    print(f"view {v}: K {int(n.sum())} tiles {gx * gy} mean {n.mean():.0f} p50 {np.median(n):.0f} "
          f"p90 {np.percentile(n, 90):.0f} p99 {np.percentile(n, 99):.0f} max {n.max()} "
          f">4096: {(n > 4096).sum()} >8192: {(n > 8192).sum()} >16384: {(n > 16384).sum()} >32768: {(n > 32768).sum()}",
          flush=True)
