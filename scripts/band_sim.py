#!/usr/bin/env python3
"""Single-GPU rehearsal of one rank of the N-GPU band pipeline (no collectives): forward on
the band, blend-backward, B2 on the rank's Gaussian slice.  Prints per-stage ms and the
step time, i.e. the per-rank compute an N-GPU run adds to its communication.
usage: band_sim.py [--world 8] [--rank 3] [--steps 20] [--config 1m_1080p]"""
import argparse
import importlib
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "3d_gaussian_splatting_amd"
gr = importlib.import_module(f"{PKG}.graphics")
sc = importlib.import_module(f"{PKG}.scene")
R = importlib.import_module(f"{PKG}.rasterizer")
native = importlib.import_module(f"{PKG}.native")
bands = importlib.import_module(f"{PKG}.bands")
bench = importlib.import_module("bench")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="1m_1080p")
    args = ap.parse_args()
    cfg = bench.CONFIGS[args.config]
    P, W, H, D = cfg["P"], cfg["W"], cfg["H"], cfg["D"]
    dev = torch.device("cuda", 0)
    cam = gr.synthetic_camera(W, H)
    scene = sc.make_scene(cam, P, max_sh_degree=max(D, 0), seed=0)
    t = lambda a: torch.tensor(a, device=dev)
    inputs = dict(means3D=t(scene.means3D), opacities=t(scene.opacities), scales=t(scene.scales),
                  rotations=t(scene.rotations), sh_dc=t(scene.sh_dc), sh_rest=t(scene.sh_rest))
    dpix = t(sc.make_dL_dpix(cam, seed=1))
    rast = R.CAbiRasterizer(dev)
    gy = cam.grid[1]
    band = bands.band_rows(gy, args.world, args.rank)
    g0, g1 = bands.gaussian_slice(P, args.world, args.rank)

    def step():
        st = rast.forward(cam, **inputs, sh_degree=D, tile_rows=band, band_only=True)
        g2 = rast.backward_blend(st, dpix)
        return st, rast.backward_preprocess_range(st, g0, g1, g2[g0:g1])

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    native.profile_enable()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    stages = native.profile_read()
    native.profile_enable(0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        st, _ = step()
    torch.cuda.synchronize()
    ms = 1e3 * (time.perf_counter() - t0) / args.steps
    print(json.dumps({"world": args.world, "rank": args.rank, "band_tile_rows": band, "ms_per_step": round(ms, 4),
                      "candidates": st.buffers.num_ranked, "num_rendered": st.num_rendered,
                      "stage_ms": {k: round(v / args.steps, 4) for k, (v, n) in stages.items() if n}}))


if __name__ == "__main__":
    main()
