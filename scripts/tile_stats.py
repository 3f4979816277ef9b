#!/usr/bin/env python3
"""Per-tile list lengths n F6 termination indices and B1 chunk tables (GSR_VIEW_RANGES / GSR_VIEW_TERM) of the
bench workload, saved for the B1 chunking analysis (how many checkpoints each chunking rule
writes and how long its longest chunk is).  usage: tile_stats.py OUT.npz [--config 1m_1080p]"""
import argparse
import importlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "3d_gaussian_splatting_amd"
gr = importlib.import_module(f"{PKG}.graphics")
sc = importlib.import_module(f"{PKG}.scene")
R = importlib.import_module(f"{PKG}.rasterizer")
native = importlib.import_module(f"{PKG}.native")
bench = importlib.import_module("bench")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--config", default="1m_1080p", choices=sorted(bench.CONFIGS))
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = bench.CONFIGS[args.config]
    cam = gr.synthetic_camera(cfg["W"], cfg["H"])
    s = sc.make_scene(cam, cfg["P"], max_sh_degree=cfg["D"], seed=0)
    t = lambda a: torch.tensor(a, device=dev)
    st = R.CAbiRasterizer(dev).forward(cam, t(s.means3D), t(s.opacities), scales=t(s.scales), rotations=t(s.rotations),
                                       sh_dc=t(s.sh_dc), sh_rest=t(s.sh_rest), sh_degree=cfg["D"])
    gx, gy = cam.grid
    ranges = st.view(native.VIEW_RANGES, torch.int32, 2 * gx * gy).cpu().numpy().reshape(-1, 2)
    table = st.view(native.VIEW_TERM, torch.int32, native.TERM_STRIDE * gx * gy).cpu().numpy().view(np.uint32)
    table = table.reshape(-1, native.TERM_STRIDE)
    term = table[:, 0].astype(np.int64)
    n = ranges[:, 1] - ranges[:, 0]
    chunks = 1 + (table[:, 1:] != 0xFFFFFFFF).sum(1)
    np.savez(args.out, n=n, term=term, table=table, grid=np.array([gx, gy]))
    print(f"B1 chunks per tile: mean {chunks.mean():.2f} max {chunks.max()}  checkpoint bytes "
          f"{int((chunks - 1).sum()) * 4096}")
    # F6 / B1 give XCD x (blocks b with b % 8 == x) a contiguous tile range (xcd_tile): the work
    # of each XCD's range (terminated records), against an interleaved tile -> XCD assignment
    T = gx * gy
    q, r = T // 8, T % 8
    starts = [x * (q + 1) if x < r else r * (q + 1) + (x - r) * q for x in range(8)] + [T]
    contig = np.array([term[starts[x]:starts[x + 1]].sum() for x in range(8)], np.float64)
    inter = np.array([term[x::8].sum() for x in range(8)], np.float64)
    print(f"XCD work (sum of term): contiguous max/mean {contig.max() / contig.mean():.3f}, "
          f"interleaved max/mean {inter.max() / inter.mean():.3f}")
    print(f"tiles {gx * gy}  n: mean {n.mean():.0f} p50 {np.median(n):.0f} p99 {np.percentile(n, 99):.0f} "
          f"max {n.max()}  term: mean {term.mean():.0f} p50 {np.median(term):.0f} p99 {np.percentile(term, 99):.0f} "
          f"max {term.max()}")


if __name__ == "__main__":
    main()
