#!/usr/bin/env python3
"""Interleaved A/B timing of kernel variants in ONE process (cdna guide rule 24).

    python scripts/ablate.py --var GSR_FWD_VARIANT=0,1 --var GSR_BWD_VARIANT=0,1 [--rounds 6]

For each round and each setting, runs `iters` forward+backward steps of the bench workload
and records per-stage milliseconds from the library's HIP-event stage profiler.
Prints median / min per (variable, value, stage).
"""
import argparse
import importlib
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
gr = importlib.import_module("3d_gaussian_splatting_amd.graphics")
sc = importlib.import_module("3d_gaussian_splatting_amd.scene")
R = importlib.import_module("3d_gaussian_splatting_amd.rasterizer")
native = importlib.import_module("3d_gaussian_splatting_amd.native")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--var", action="append", default=[])
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--P", type=int, default=1_000_000)
    ap.add_argument("--W", type=int, default=1920)
    ap.add_argument("--H", type=int, default=1080)
    args = ap.parse_args()
    cam = gr.synthetic_camera(args.W, args.H)
    s = sc.make_scene(cam, args.P, max_sh_degree=3, seed=0)
    dev = torch.device("cuda")
    t = lambda a: torch.tensor(a, device=dev)
    inputs = dict(means3D=t(s.means3D), opacities=t(s.opacities), scales=t(s.scales), rotations=t(s.rotations),
                  sh_dc=t(s.sh_dc), sh_rest=t(s.sh_rest))
    dpix = t(sc.make_dL_dpix(cam, seed=1))
    rast = R.CAbiRasterizer(dev)
    settings = []
    for v in args.var:
        name, vals = v.split("=")
        settings += [(name, x) for x in vals.split(",")]
    res = {}
    ref = None
    for rnd in range(args.rounds):
        for name, val in settings:
            os.environ[name] = val
            st = rast.forward(cam, **inputs, sh_degree=3)  # warm
            g = rast.backward(st, dpix)
            torch.cuda.synchronize()
            if rnd == 0:
                out = (st.color.clone(), g["means3D"].clone())
                if ref is None:
                    ref = out
                else:
                    dc = float((out[0] - ref[0]).abs().max())
                    dg = float((out[1] - ref[1]).norm() / ref[1].norm())
                    print(f"check {name}={val}: max|dcolor|={dc:.3g} rel dmeans3D={dg:.3g}", flush=True)
            native.profile_enable()
            for _ in range(args.iters):
                st = rast.forward(cam, **inputs, sh_degree=3)
                rast.backward(st, dpix)
            torch.cuda.synchronize()
            prof = native.profile_read()
            for stage, (ms, n) in prof.items():
                if n:
                    res.setdefault((name, val, stage), []).append(ms / args.iters)
            os.environ.pop(name, None)
    summary = {}
    for (name, val, stage), xs in sorted(res.items()):
        summary[f"{name}={val}:{stage}"] = (round(statistics.median(xs), 4), round(min(xs), 4))
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
