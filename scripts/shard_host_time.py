#!/usr/bin/env python3
"""Host cost of one multi-GPU step (bands.ShardStep.step: every ctypes call, allocation and
collective launch of a rank), measured on a single-rank RCCL group: the wall time for step()
to return (no synchronisation inside) against the GPU time of the same step.  The host cost is
what each rank pays per step whatever N is; at N = 8 the per-rank GPU work is ~1/8 of this
one, so a host cost near that figure makes the real run host-bound.
--impl cpp times the C++ step instead (`_gsr_torch.ShardStep` over a world-1 RCCL exchange,
graph replay: the benchmark's multi-GPU path).
usage: shard_host_time.py [--config 1m_1080p] [--steps 20] [--impl python|cpp]"""
import argparse
import importlib
import json
import os
import socket
import sys
import time

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
    ap.add_argument("--config", default="1m_1080p", choices=sorted(bench.CONFIGS))
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--cprofile", action="store_true", help="print the host hot spots of step()")
    ap.add_argument("--impl", default="python", choices=("python", "cpp"))
    args = ap.parse_args()
    if args.impl == "cpp":
        return cpp_main(args)
    import torch.distributed as dist
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    cfg = bench.CONFIGS[args.config]
    cam = gr.synthetic_camera(cfg["W"], cfg["H"])
    s = sc.make_scene(cam, cfg["P"], max_sh_degree=cfg["D"], seed=0)
    t = lambda a: torch.tensor(a, device=dev)
    inputs = dict(means3D=t(s.means3D), opacities=t(s.opacities), scales=t(s.scales), rotations=t(s.rotations),
                  sh_dc=t(s.sh_dc), sh_rest=t(s.sh_rest))
    dpix = t(sc.make_dL_dpix(cam, seed=1))
    step = bands.ShardStep(R.ShardRasterizer(dev), cam, inputs, cfg["D"], dist).plan()
    for _ in range(3):
        step.step(dpix)
    torch.cuda.synchronize()
    host, gpu = [], []
    for _ in range(args.steps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        h0 = time.perf_counter()
        step.step(dpix)
        host.append((time.perf_counter() - h0) * 1e3)
        e1.record()
        torch.cuda.synchronize()
        gpu.append(e0.elapsed_time(e1))
    if args.cprofile:
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(args.steps):
            step.step(dpix)
        pr.disable()
        torch.cuda.synchronize()
        pstats.Stats(pr, stream=sys.stderr).sort_stats("tottime").print_stats(25)
    host.sort()
    gpu.sort()
    print(json.dumps({"config": args.config, "host_ms_median": round(host[len(host) // 2], 4),
                      "gpu_ms_median": round(gpu[len(gpu) // 2], 4), "steps": args.steps}))
    dist.destroy_process_group()


def cpp_main(args):
    native = importlib.import_module(f"{PKG}.native")
    ext = native.load_torch_ext()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = bench.CONFIGS[args.config]
    cam = gr.synthetic_camera(cfg["W"], cfg["H"])
    s = sc.make_scene(cam, cfg["P"], max_sh_degree=cfg["D"], seed=0)
    t = lambda a: torch.tensor(a, device=dev)
    inputs = dict(means3D=t(s.means3D), opacities=t(s.opacities), scales=t(s.scales), rotations=t(s.rotations),
                  sh_dc=t(s.sh_dc), sh_rest=t(s.sh_rest))
    dpix = t(sc.make_dL_dpix(cam, seed=1))
    ex = ext.rccl_exchange(ext.rccl_unique_id(), 0, 1)
    step = ext.ShardStep(ex, R.ext_camera(cam), inputs, cfg["D"], graph=True)
    step.plan()
    for _ in range(3):
        step.step(dpix)
    torch.cuda.synchronize()
    assert step.graph_active
    host, gpu = [], []
    for _ in range(args.steps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        h0 = time.perf_counter()
        step.step(dpix)
        host.append((time.perf_counter() - h0) * 1e3)
        e1.record()
        torch.cuda.synchronize()
        gpu.append(e0.elapsed_time(e1))
    step.check()
    host.sort()
    gpu.sort()
    print(json.dumps({"config": args.config, "impl": "cpp (graph replay, RCCL world 1)",
                      "host_ms_median": round(host[len(host) // 2], 4),
                      "gpu_ms_median": round(gpu[len(gpu) // 2], 4), "steps": args.steps}))


if __name__ == "__main__":
    main()
