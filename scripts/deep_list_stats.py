#!/usr/bin/env python3
"""Deep tile lists after an opacity reset: the configs[4] scene at ~6M Gaussians,
trained for a few iterations, rendered from one view before and after `reset_opacity`.  Prints,
per state, the F6 / B1 stage times (HIP events, median of 5) and the per-tile distribution of
list length n, termination index tend and B1 chunks -- whether the blend kernels are bound by
their total work or by the serial chain of the deepest tiles.

usage: python scripts/deep_list_stats.py [--gt N] [--init N] [--size WxH] [--iters N]
"""
import argparse
import importlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "3d_gaussian_splatting_amd"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gt", type=int, default=8_000_000)
    ap.add_argument("--init", type=int, default=6_000_000)
    ap.add_argument("--size", default="1280x832")
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    L = importlib.import_module(f"{PKG}.train_loop")
    T = importlib.import_module(f"{PKG}.trainer")
    native = importlib.import_module(f"{PKG}.native")
    sc = importlib.import_module(f"{PKG}.scene")
    dev = torch.device("cuda", 0)
    W, H = (int(v) for v in a.size.split("x"))
    scene = L.synthetic_scene(a.gt, a.init, 4, W, H, seed=0, device=dev, texture=1.0, gt_scale=0.012)
    tr = T.GaussianTrainer.from_point_cloud(scene.points, scene.colors, 3, spatial_lr_scale=scene.extent, device=dev)
    tr.setup(T.OptimizationParams())
    for it in range(1, a.iters + 1):
        tr.step(it, scene.cams[it % 4], scene.gts[it % 4], densify=False)
    torch.cuda.synchronize()
    cam = scene.cams[0]
    gx, gy = cam.grid
    tiles = gx * gy
    dpix = torch.tensor(sc.make_dL_dpix(cam, seed=1), device=dev)

    def measure(tag):
        reps = []
        for _ in range(6):
            native.profile_enable()
            st = tr.render(cam)
            tr.rast.backward(st, dpix)
            torch.cuda.synchronize()
            reps.append(native.profile_read())
            native.profile_enable(0)
        stage = {k: round(float(np.median([r[k][0] for r in reps[1:]])), 4) for k in reps[0] if reps[0][k][1]}
        rng = st.view(native.VIEW_RANGES, torch.int32, 2 * tiles).cpu().numpy().reshape(-1, 2).astype(np.int64)
        n = rng[:, 1] - rng[:, 0]
        term = st.view(native.VIEW_TERM, torch.int32, native.TERM_STRIDE * tiles).cpu().numpy()
        term = term.view(np.uint32).reshape(tiles, native.TERM_STRIDE)
        tend = np.minimum(term[:, 0].astype(np.int64), n)
        chunks = 1 + (term[:, 1:] != 0xFFFFFFFF).sum(axis=1)
        pct = lambda x: {p: int(np.percentile(x, p)) for p in (50, 90, 99)} | {"max": int(x.max()), "mean": round(float(x.mean()), 1)}
        # the longest chunk of each tile, in list entries (B1's serial walk)
        starts = np.concatenate([np.zeros((tiles, 1), np.int64), term[:, 1:].astype(np.int64)], axis=1)
        starts = np.where(starts == 0xFFFFFFFF, -1, starts)
        longest = np.zeros(tiles, np.int64)
        for t in np.argsort(-tend)[:64]:
            s = sorted(x for x in starts[t] if x >= 0) + [int(tend[t])]
            longest[t] = max(s[i + 1] - s[i] for i in range(len(s) - 1)) if len(s) > 1 else int(tend[t])
        out = {"state": tag, "K": int(st.num_rendered), "points": int(tr.num_points), "stage_ms": stage,
               "n": pct(n), "tend": pct(tend), "tend_sum": int(tend.sum()), "chunks": pct(chunks),
               "tiles_32_chunks": int((chunks == native.TERM_STRIDE).sum()),
               "deepest_tend": [int(x) for x in np.sort(tend)[-8:]],
               "longest_chunk_top64": int(longest.max()),
               "opacity_mean": round(float(torch.sigmoid(tr.params["opacity"]).mean()), 4)}
        print(json.dumps(out), flush=True)

    measure("trained")
    tr.reset_opacity()
    measure("after_reset")


if __name__ == "__main__":
    main()
