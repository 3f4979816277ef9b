#!/usr/bin/env python3
"""Single-GPU rehearsal of the N-GPU path (bands.simulate_ranks: every rank's calls in one
process, collectives replaced by block copies).  For each N it times every rank's compute --
gsr_shard_forward (F1 + splat pack), gsr_band_forward (unpack + F2..F6), gsr_band_backward
(B1 + per-splat gather), gsr_shard_backward (B2 with the band sum fused) -- with HIP events on the
launch stream, median over --steps runs, and reports the slowest rank's total: the per-step
compute an N-GPU run adds to its communication.  Also the bytes each rank moves per step
(splat blocks out, gradient blocks back, its image band), for the xGMI estimate in DESIGN §7.
usage: band_sim.py [--worlds 1,2,4,8] [--steps 5] [--config 5m_1080p] [--cpp]

--cpp: the C++ gsr::ShardStep instead (what bench.py --gpus N runs): N ranks in one process, one
host thread each, over an in-process exchange (ext.LocalGroup: device copies between the ranks'
buffers); after two live steps every rank's WHOLE step -- the four C-ABI calls, the glue around
the exchanges (gsr_band_publish / gsr_gather_finish), the exchange-sized copies and the hipGraph
replay -- is timed alone on the GPU, with the copies ("with_copies") and without the all-to-all copies
("compute": the image all-gather's copy stays, overlapped with B1 on the side stream as RCCL's
would be), and its image is checked against the single-GPU render."""
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
gr = importlib.import_module(f"{PKG}.graphics")
sc = importlib.import_module(f"{PKG}.scene")
R = importlib.import_module(f"{PKG}.rasterizer")
bands = importlib.import_module(f"{PKG}.bands")
bench = importlib.import_module("bench")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--config", default="5m_1080p", choices=sorted(bench.CONFIGS))
    ap.add_argument("--no-single", action="store_true", help="skip the single-GPU reference step (kernel traces)")
    ap.add_argument("--lib", default=None, help="an experimental libgsr_hip.so (_build.build_variant)")
    ap.add_argument("--cpp", action="store_true", help="time the C++ ShardStep per rank (see above)")
    ap.add_argument("--cpp-graph", type=int, default=1, help="--cpp: replay each rank's step as a hipGraph (1) "
                                                            "or eagerly (0)")
    args = ap.parse_args()
    if args.lib:
        importlib.import_module(f"{PKG}.native").HIP_LIB = os.path.abspath(args.lib)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = bench.CONFIGS[args.config]
    P, W, H, D = cfg["P"], cfg["W"], cfg["H"], cfg["D"]
    cam = gr.synthetic_camera(W, H)
    s = sc.make_scene(cam, P, max_sh_degree=D, seed=0)
    t = lambda a: torch.tensor(a, device=dev)
    inputs = dict(means3D=t(s.means3D), opacities=t(s.opacities), scales=t(s.scales), rotations=t(s.rotations),
                  sh_dc=t(s.sh_dc), sh_rest=t(s.sh_rest))
    del s
    dpix = t(sc.make_dL_dpix(cam, seed=1))
    rast = R.ShardRasterizer(dev)
    single = R.CAbiRasterizer(dev)
    # the single-GPU step for reference (same timing method)
    K0 = 0 if args.no_single else single.forward(cam, **inputs, sh_degree=D).num_rendered
    cap = bands.round_up(int(K0 * 1.1) + 1)
    ref = []
    for i in range(0 if args.no_single else args.steps + 2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        st = single.forward(cam, **inputs, sh_degree=D, max_rendered=cap)
        single.backward(st, dpix)
        e1.record()
        torch.cuda.synchronize()
        if i >= 2:
            ref.append(e0.elapsed_time(e1))
    one_gpu = float(np.median(ref)) if ref else float("nan")
    print(json.dumps({"config": args.config, "world": 1, "path": "single-GPU gsr_forward + gsr_backward",
                      "ms_per_step": round(one_gpu, 4)}), flush=True)
    if args.cpp:
        for world in [int(w) for w in args.worlds.split(",")]:
            cpp_rehearsal(args, cam, inputs, D, dpix, world, one_gpu, None if args.no_single else st.color)
        return
    for world in [int(w) for w in args.worlds.split(",")]:
        plan = None
        runs = []
        for i in range(args.steps + 1):
            times = {}

            def timer(name, r, fn):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                out = fn()
                e1.record()
                times.setdefault(r, []).append((name, e0, e1))
                return out

            img, g, plan = bands.simulate_ranks(rast, cam, inputs, D, world, dpix, timer=timer,
                                                rows=None if plan is None else plan["rows"])
            torch.cuda.synchronize()
            if i >= 1:
                runs.append({r: {n: a.elapsed_time(b) for n, a, b in v} for r, v in times.items()})
        per_rank = {r: {n: float(np.median([run[r][n] for run in runs])) for n in runs[0][r]} for r in runs[0]}
        totals = {r: sum(v.values()) for r, v in per_rank.items()}
        slow = max(totals, key=totals.get)
        pc = plan["pair_cap"]
        band_px = [(min(plan["rows"][b + 1] * 16, H) - plan["rows"][b] * 16) * W for b in range(world)]
        print(json.dumps({
            "config": args.config, "world": world, "rows": plan["rows"], "pair_cap": pc,
            "band_capacity": plan["capacity"], "band_instances": plan["band_instances"],
            "splats_per_pair_max": max(int(sh.counts.max()) for sh in plan["shards"]),
            "rank_ms": {r: round(v, 4) for r, v in totals.items()},
            "slowest_rank": slow, "slowest_rank_stages_ms": {n: round(v, 4) for n, v in per_rank[slow].items()},
            "slowest_rank_ms": round(totals[slow], 4), "single_gpu_ms": round(one_gpu, 4),
            "compute_speedup": round(one_gpu / totals[slow], 3),
            "bytes_per_rank": {"splats_out": world * (pc + 1) * 64, "grads_back": world * pc * 48,
                               "image_band": 12 * max(band_px)},
        }), flush=True)


def cpp_rehearsal(args, cam, inputs, D, dpix, world, one_gpu, color):
    """Every rank's whole C++ step (gsr::ShardStep) timed alone, after live steps in threads."""
    ext = importlib.import_module(f"{PKG}.native").load_torch_ext()
    grp = ext.LocalGroup(world)
    exs = [ext.local_exchange(grp, r) for r in range(world)]
    ecam = R.ext_camera(cam)
    steps = [ext.ShardStep(exs[r], ecam, inputs, D, graph=False) for r in range(world)]
    ext.run_ranks_plan(steps)
    ext.run_ranks_steps(steps, dpix, 2)  # live: every rank's collectives with the others
    torch.cuda.synchronize()
    out = {"config": args.config, "world": world,
           "impl": "C++ gsr::ShardStep, in-process exchange, " + ("graph replay" if args.cpp_graph else "eager steps"),
           "rows": list(steps[0].rows), "pair_cap": steps[0].pair_cap, "band_capacity": steps[0].capacity,
           "band_instances": list(steps[0].band_instances)}
    for mode in ("with_copies", "compute"):
        rank_ms, equal, graphs = {}, [], []
        for r in range(world):
            ext.local_exchange_set_replay(exs[r], True, mode == "with_copies")
            steps[r].set_graph(False)  # drop a graph captured in the other mode
            steps[r].set_graph(args.cpp_graph == 1)
            for _ in range(3):  # eager, capture, replay
                img, g, radii = steps[r].step(dpix)
            torch.cuda.synchronize()
            times = []
            for _ in range(args.steps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                img, g, radii = steps[r].step(dpix)
                e1.record()
                torch.cuda.synchronize()
                times.append(e0.elapsed_time(e1))
            steps[r].check()
            rank_ms[r] = float(np.median(times))
            graphs.append(bool(steps[r].graph_active))
            if color is not None:
                equal.append(bool(torch.equal(img, color)))
        slow = max(rank_ms, key=rank_ms.get)
        out[mode] = {"rank_ms": {r: round(v, 4) for r, v in rank_ms.items()}, "slowest_rank": slow,
                     "slowest_rank_ms": round(rank_ms[slow], 4), "graph_replay": all(graphs),
                     "compute_speedup": round(one_gpu / rank_ms[slow], 3) if one_gpu == one_gpu else None}
        if equal:
            out[mode]["image_equals_single_gpu"] = all(equal)
    out["single_gpu_ms"] = round(one_gpu, 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
