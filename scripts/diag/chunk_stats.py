#!/usr/bin/env python3
"""Chunk-table statistics of one full-image forward (GSR_VIEW_TERM): per tile the termination
index, the number of B1 chunks F6 opened, and the records in each chunk.  A band launch holds
the same tile lists as the full image, so the per-band maxima below are the critical paths of
a band's F6 (records to termination of its deepest tile) and B1 (its longest chunk).
usage: chunk_stats.py [--config 1m_1080p] [--world 8]"""
import argparse
import importlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
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
    ap.add_argument("--config", default="1m_1080p", choices=sorted(bench.CONFIGS))
    ap.add_argument("--world", type=int, default=8)
    args = ap.parse_args()
    cfg = bench.CONFIGS[args.config]
    dev = torch.device("cuda", 0)
    cam = gr.synthetic_camera(cfg["W"], cfg["H"])
    s = sc.make_scene(cam, cfg["P"], max_sh_degree=cfg["D"], seed=0)
    t = lambda a: torch.tensor(a, device=dev)
    st = R.CAbiRasterizer(dev).forward(cam, t(s.means3D), t(s.opacities), t(s.scales), t(s.rotations),
                                       t(s.sh_dc), t(s.sh_rest), sh_degree=cfg["D"])
    gx, gy = (cam.width + 15) // 16, (cam.height + 15) // 16
    tiles = gx * gy
    term = st.view(native.VIEW_TERM, torch.int32, tiles * native.TERM_STRIDE).cpu().numpy().view(np.uint32)
    term = term.reshape(tiles, native.TERM_STRIDE).astype(np.int64)
    rng = st.view(native.VIEW_RANGES, torch.int32, 2 * tiles).cpu().numpy().view(np.uint32).reshape(-1, 2)
    n = (rng[:, 1].astype(np.int64) - rng[:, 0])
    tend = np.minimum(term[:, 0], n)
    starts = term[:, 1:]
    nck = (starts != 0xFFFFFFFF).sum(1)
    longest = np.zeros(tiles, np.int64)
    last = np.zeros(tiles, np.int64)
    for i in range(tiles):
        b = [0] + [int(x) for x in starts[i, :nck[i]]] + [int(tend[i])]
        lens = np.diff(b)
        longest[i] = lens.max() if len(lens) else 0
        last[i] = lens[-1] if len(lens) else 0
    hist = np.zeros(gy, np.int64)
    for ty in range(gy):
        hist[ty] = n[ty * gx:(ty + 1) * gx].sum()
    rows = bands.balance_bands(hist, args.world)
    per_band = []
    for b in range(args.world):
        sl = slice(rows[b] * gx, rows[b + 1] * gx)
        per_band.append({"rows": [int(rows[b]), int(rows[b + 1])], "max_term": int(tend[sl].max()),
                         "mean_term": round(float(tend[sl].mean()), 1), "max_chunk_records": int(longest[sl].max()),
                         "tiles_at_cap": int((nck[sl] == native.TERM_STRIDE - 1).sum()),
                         "max_last_chunk": int(last[sl].max())})
    print(json.dumps({"config": args.config, "tiles": tiles, "K": int(n.sum()),
                      "term": {"max": int(tend.max()), "p99": float(np.percentile(tend, 99)), "mean": float(tend.mean())},
                      "chunks": {"max": int(nck.max()), "mean": round(float(nck.mean()), 2),
                                 "tiles_at_cap": int((nck == native.TERM_STRIDE - 1).sum())},
                      "longest_chunk_records": {"max": int(longest.max()), "p99": float(np.percentile(longest, 99)),
                                                "mean": round(float(longest.mean()), 1)},
                      "world": args.world, "bands": per_band}))


if __name__ == "__main__":
    main()
