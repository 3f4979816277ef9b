#!/usr/bin/env python3
"""Benchmark: forward+backward of the MI355X 3DGS rasterizer (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 1m_1080p|100k_800|5m_1080p]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One step = gsr_forward + gsr_backward (through the C ABI) of the whole synthetic scene:
1M Gaussians, 1920x1080, SH degree 3 (BASELINE configs[2], the roofline run; inputs already
resident in HBM).  The binning is sized from the first (untimed) forward's K with 10 %
headroom (gsr_raster_settings.max_rendered), so no step waits on a host read.  N > 1 (one
process per GPU, RCCL): the Gaussian-sharded x tile-row-band split of bands.ShardStep -- F1 on
the rank's Gaussian shard, all-to-all of the projected splats to the bands, band binning +
blend, asynchronous all-gather of the band images (overlaps B1), B1 on the band, all-to-all of
the splats' 2D gradients back, B2 on the shard.  The whole image is rendered once per step for
the job, so value = steps/s of the job ("scaling": "strong").  Rank 0 prints ONE JSON line.

roofline: the dominant kernel's algorithmic HBM bytes (SURVEY §8d formulas) per
launch / its mean launch time from HIP events recorded on the launch stream over the timed
region (gsr_profile_*), against 8.0 TB/s.  `traffic` / `valu_issue` come from the committed
rocprofv3 PMC passes (profiles/pmc_traffic.json) and are dropped unless those passes were of
this workload AND of this build of libgsr_hip.so (source stamp).  cpu_baseline: the CPU oracle
(oracle/, a C port of the same algorithm) timed on this host's cores, median of 3
forward+backward iterations of the same workload after one warm-up (rank 0, N = 1), which also
gives the PSNR / gradient error of the GPU result.
"""
from __future__ import annotations

import argparse
import importlib
import json
import math
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
PKG = "3d_gaussian_splatting_amd"
gr = importlib.import_module(f"{PKG}.graphics")
sc = importlib.import_module(f"{PKG}.scene")
R = importlib.import_module(f"{PKG}.rasterizer")
native = importlib.import_module(f"{PKG}.native")
bands = importlib.import_module(f"{PKG}.bands")

WARMUP_FLOOR_S = 0.5  # untimed warm-up seconds before the timed steps (render mode)

CONFIGS = {
    "1k_256": dict(P=1_000, W=256, H=256, D=0),
    "100k_800": dict(P=100_000, W=800, H=800, D=3),
    "1m_1080p": dict(P=1_000_000, W=1920, H=1080, D=3),
    "5m_1080p": dict(P=5_000_000, W=1920, H=1080, D=3),
    # the training loop's image size (BASELINE configs[4]) at two densities: A/B cases for the
    # binning choice (global depth pre-sort vs row-bucketed binning), not bench lines
    "3m_1280x832": dict(P=3_000_000, W=1280, H=832, D=3),
    "6m_1280x832": dict(P=6_000_000, W=1280, H=832, D=3),
}
BASELINE_METRIC = "forward+backward iters/s at 1080p, 1M Gaussians; PSNR vs CPU ref"  # BASELINE.json


def config_label(name: str) -> str:
    c = CONFIGS[name]
    size = "1080p" if (c["W"], c["H"]) == (1920, 1080) else f"{c['W']}x{c['H']}"
    n = f"{c['P'] // 1_000_000}M" if c["P"] % 1_000_000 == 0 else f"{c['P'] // 1000}k"
    return f"{size}, {n} Gaussians"


def config_metric(name: str) -> str:
    """BASELINE.json's metric string for its config (1m_1080p); the same metric named after the
    workload for the others (parity-test sizes and configs[3]'s 5M scene)."""
    return f"forward+backward iters/s at {config_label(name)}; PSNR vs CPU ref"


HBM_PEAK_GBS = 8000.0  # MI355X spec, /opt/skills/guides/MI355X_MICROARCH.md
# wave64 VALU issue peak: 256 CUs x 4 SIMD-32 units, one wave64 op per 2 cycles per SIMD at
# 2.4 GHz (MI355X_MICROARCH constants table, `v_fma_f32 (wave64) 2 cyc (SIMD-32)`).  This spec
# rate is the only issue ceiling reported (a measured FMA-stream rate is not a ceiling: the
# blend kernels exceed it with their mix of moves, selects and DPP adds).
VALU_ISSUE_PER_S = 256 * 4 * 2.4e9 / 2
# SURVEY §8d secondary bound for F6 + B1, from the ISA: the wave64 VALU
# instructions of the kernels' per-stripe loop bodies in the shipped gfx950 code x the
# number of times the culled loops must run them, counted exactly by the CPU oracle
# (gsr_oracle.State.blend_work: the kernels' box + ellipse stripe masks, exact per-pixel
# termination -- lower bounds of the kernels' own counts) -- over the spec issue peak.  Per-record
# set-up, batch loads, reductions and loop control are left out, so floor / measured is the share
# of the blend time the unavoidable arithmetic would take at full issue rate.
F6_VISIT_VALU = 32        # blend_forward_kernel<2>: one wave's visit of a record, its two stripes
B1_STRIPE_VALU = 12       # blend_backward_kernel<4>: one stripe evaluation (exp, alpha, T update)
B1_CONTRIB_VALU = 16      # ... plus the contribution block when a lane of the stripe contributes


ALG_STAGES = ("preprocess", "scan", "duplicate", "tile_sort", "finalize", "blend_fwd", "blend_bwd",
              "preprocess_bwd")


def algorithmic_bytes(P, V, K, pix, tiles, M):
    """SURVEY §8d compulsory traffic per stage (bytes), M = (D+1)^2 SH coefficients."""
    return {
        "preprocess": P * (44 + 8) + V * (12 * M + 40),
        "scan": P * 8,
        "duplicate": V * 20 + K * 12,
        "tile_sort": K * 24,
        "finalize": K * 8 + tiles * 8,
        "blend_fwd": tiles * 8 + K * 40 + pix * 20,
        "blend_bwd": tiles * 8 + K * 40 + pix * 20 + V * 36,
        "preprocess_bwd": V * (80 + 12 * M) + P * (60 + 12 * M),
    }


def stage_bytes(P, V, K, pix, tiles, M):
    """Algorithmic bytes of EVERY timed stage (the §8d table plus the two stages it folds into
    others): the per-tile depth sort reads and writes each instance's gid and gathers its 4-B
    depth key (12 B per instance); the per-Gaussian gather reads each instance's 36-B partial and
    writes a 48-B grad2d row per visible Gaussian."""
    b = algorithmic_bytes(P, V, K, pix, tiles, M)
    b["depth_sort"] = K * 12
    b["gather_grad2d"] = K * 36 + V * 48
    return b


def lib_stamp() -> str | None:
    """Source stamp of the loaded libgsr_hip.so (sha256 of its sources + flags, _build.py)."""
    path = native.hip_library_path() + ".stamp"
    return open(path).read().strip() if os.path.exists(path) else None


def pmc_record(kernel_prefix, workload):
    """Per-launch PMC figures of `kernel_prefix` (HBM bytes, VALU instructions) from the
    committed rocprofv3 passes (profiles/pmc_traffic.json, written by
    scripts/pmc_summary.py --traffic), or {} when those passes were of another workload or of
    another build of the library (their lib_stamp differs from the loaded one)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return {}
    with open(path) as fh:
        data = json.load(fh)
    if data.get("workload") != workload or data.get("lib_stamp") != lib_stamp():
        return {}
    for name, rec in data.get("kernels", {}).items():
        if name.startswith(kernel_prefix):
            return rec
    return {}


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


class CppShard:
    """bench's view of the C++ multi-GPU step (ext.ShardStep): the same attributes bands.ShardStep
    offers the reporting code below.  Over RCCL (--dist-backend nccl, one GPU per rank, the step
    captured into a hipGraph) the unique id travels over the torch.distributed group that the
    launcher already set up; with --dist-backend gloo the exchange is the host-staged
    ext.store_exchange over that group's c10d store -- the same C++ step, ranks may share one GPU
    (the rehearsal of the driver's N-GPU line; not capturable, so every step runs eagerly)."""

    class _Band:  # num_rendered of the band (read back after the timed loop)
        def __init__(self, st):
            self._st = st

        @property
        def num_rendered(self):
            return int(self._st.band_num_rendered())

    class _Shard:
        def __init__(self, radii):
            self.radii = radii

    def __init__(self, cam, inputs, D, dist, rank, world, backend="nccl"):
        ext = native.load_torch_ext()
        if backend == "nccl":
            uid = [ext.rccl_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            self.exchange = ext.rccl_exchange(uid[0], rank, world)
        else:
            self.exchange = ext.store_exchange(dist.distributed_c10d._get_default_store(), rank, world)
        self.st = ext.ShardStep(self.exchange, R.ext_camera(cam), inputs, D, graph=True)
        self.st.plan()
        self.rank = rank
        self.rows, self.pair_cap, self.capacity = list(self.st.rows), self.st.pair_cap, self.st.capacity
        self.band_instances = list(self.st.band_instances)
        self.g0, self.g1 = self.st.g0, self.st.g1
        self.band = (self.rows[rank], self.rows[rank + 1])
        # ranks as the transport counts them: ncclCommCount of the step's communicator (RCCL), the
        # ranks that joined the exchange's store key (store)
        self.comm_world = int(self.st.exchange_world)
        self.impl = ("C++ gsr::ShardStep over RCCL, hipGraph replay" if backend == "nccl" else
                     "C++ gsr::ShardStep over a host-staged c10d store exchange (rehearsal: ranks may share a "
                     "GPU; device->host->store copies instead of RCCL's xGMI transfers, eager steps, no graph)")

    def check(self):  # every pending step's agreed overflow check (waits)
        self.st.check()

    def step(self, dpix):
        img, g, radii = self.st.step(dpix)
        return self._Band(self.st), g, self._Shard(radii)


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_or_refuse(args) -> int | None:
    """`--gpus N` means N ranks (BASELINE north_star: throughput at 1, 2, 4 and 8 GPUs).

    - Under a launcher (WORLD_SIZE set): WORLD_SIZE must equal --gpus, else exit 2.
    - No launcher and --gpus N > 1: start N ranks as ONE child process (torch.distributed.run on
      127.0.0.1, this script with the same arguments) and return its exit code.  Nothing here has
      touched the GPU (torch.cuda.device_count() does not initialise it on this image), and the
      parent only waits: no exec from a GPU process.
    - --gpus N > 1 over RCCL needs N devices: fewer visible devices exit 2 (gloo ranks may share
      one GPU: the rehearsal).
    Returns None when this process is the one to run the benchmark."""
    env_world = os.environ.get("WORLD_SIZE")
    if args.gpus < 1:
        print(f"bench.py: --gpus must be >= 1 (got {args.gpus})", file=sys.stderr)
        return 2
    if env_world is not None:
        if int(env_world) != args.gpus:
            print(f"bench.py: WORLD_SIZE={env_world} from the launcher but --gpus {args.gpus}: refusing to "
                  f"report a {env_world}-rank run as {args.gpus} GPUs", file=sys.stderr)
            return 2
        return None
    if args.gpus == 1:
        return None
    if args.mode != "render" and not args.launch_check:
        print(f"bench.py: --mode {args.mode} runs on one GPU; --gpus {args.gpus} refused", file=sys.stderr)
        return 2
    if args.dist_backend == "nccl" and not args.launch_check:
        ndev = torch.cuda.device_count()
        if ndev < args.gpus:
            print(f"bench.py: --gpus {args.gpus} over RCCL needs {args.gpus} visible GPUs, found {ndev} "
                  f"(use --dist-backend gloo to rehearse ranks sharing a GPU)", file=sys.stderr)
            return 2
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this pool (RCCL)
    return subprocess.call(cmd, env=env)


def launch_check_main(args):
    """--launch-check: each rank joins the process group (gloo, no device) and the world is counted
    by an all-reduce of ones; rank 0 prints the count as n_gpus.  Tests the launch path on a CPU."""
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    counted = 1
    if world > 1:
        dist.init_process_group("gloo")
        t = torch.ones(1, dtype=torch.int64)
        dist.all_reduce(t)
        counted = int(t.item())
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "ranks_counted": counted, "gpus_arg": args.gpus}))
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="1m_1080p", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-stage-events", action="store_true")
    ap.add_argument("--views", type=int, default=8, help="--mode views: cameras per batch")
    ap.add_argument("--iters", type=int, default=30000, help="--mode loop: training iterations")
    ap.add_argument("--loop-gt", type=int, default=4_000_000, help="--mode loop: ground-truth Gaussians")
    ap.add_argument("--loop-init", type=int, default=1_000_000, help="--mode loop: initial points")
    ap.add_argument("--loop-size", default="1280x832", help="--mode loop: image size WxH")
    ap.add_argument("--loop-views", type=int, default=128, help="--mode loop: training cameras")
    ap.add_argument("--loop-texture", type=float, default=1.0, help="--mode loop: ground-truth colour noise")
    ap.add_argument("--loop-gt-scale", type=float, default=0.012, help="--mode loop: ground-truth splat size")
    ap.add_argument("--loop-engine", default="cpp", choices=("cpp", "python"),
                    help="--mode loop: the C++ loop executable (lib/gsr_train_loop over gsr::Trainer, the "
                         "train.cpp drop-in) or the Python mirror (train_loop.train)")
    ap.add_argument("--mode", default="render", choices=("render", "train", "views", "loop"),
                    help="render: the BASELINE metric (rasterizer forward+backward); train: one full "
                         "training iteration (activations, render, L1+D-SSIM loss, backward, "
                         "densification statistics, fused Adam), SURVEY §8f")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL, one GPU per rank) or gloo (rehearsal: ranks may share a GPU)")
    ap.add_argument("--dist-impl", default="cpp", choices=("cpp", "python"),
                    help="N > 1: the C++ gsr::ShardStep (cpp: over RCCL with hipGraph replay, or with "
                         "--dist-backend gloo over the host-staged store exchange), or bands.ShardStep over "
                         "torch.distributed (python)")
    ap.add_argument("--exact-k", action="store_true",
                    help="size the binning from K every step (one host read per forward) instead of a bound")
    ap.add_argument("--lib", default=None, help="load this libgsr_hip.so instead of the in-tree one "
                                                  "(experimental builds: _build.build_variant)")
    ap.add_argument("--launch-check", action="store_true",
                    help="launcher plumbing only: start the --gpus ranks, join the process group, count the "
                         "ranks with one all-reduce, print that as a JSON line and exit (no GPU work)")
    args = ap.parse_args()
    rc = launch_or_refuse(args)
    if rc is not None:
        sys.exit(rc)
    if args.lib:
        native.HIP_LIB = os.path.abspath(args.lib)
    if args.launch_check:
        return launch_check_main(args)
    if args.mode == "train":
        return train_main(args)
    if args.mode == "views":
        return views_main(args)
    if args.mode == "loop":
        return loop_main(args)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", local_rank % max(ndev, 1))
    torch.cuda.set_device(dev)
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)

    cfg = CONFIGS[args.config]
    P, W, H, D = cfg["P"], cfg["W"], cfg["H"], cfg["D"]
    cam = gr.synthetic_camera(W, H)
    scene = sc.make_scene(cam, P, max_sh_degree=max(D, 0), seed=0)
    dpix_np = sc.make_dL_dpix(cam, seed=1)
    t = lambda a: torch.tensor(a, device=dev)
    inputs = dict(means3D=t(scene.means3D), opacities=t(scene.opacities), scales=t(scene.scales),
                  rotations=t(scene.rotations), sh_dc=t(scene.sh_dc), sh_rest=t(scene.sh_rest))
    dpix = t(dpix_np)
    gx, gy = cam.grid
    if world > 1 and args.dist_impl == "cpp":
        # the C++ step (csrc/torch/gsr_shard.h) over RCCL, captured into a hipGraph on its first
        # step and replayed: one graph launch per rank and step (gloo: the same step over the
        # host-staged store exchange)
        plan = CppShard(cam, inputs, D, dist, rank, world, backend=args.dist_backend)
        band = plan.band

        def step():
            return plan.step(dpix)
    elif world > 1:
        rast = R.ShardRasterizer(dev)
        plan = bands.ShardStep(rast, cam, inputs, D, dist).plan()
        band = plan.band

        def step():
            img, g, sh, st = plan.step(dpix)
            return st, g, sh
    else:
        rast = R.CAbiRasterizer(dev)
        K0 = rast.forward(cam, **inputs, sh_degree=D).num_rendered  # sizes the binning once
        cap = 0 if args.exact_k else bands.round_up(int(K0 * 1.1) + 1)

        def step():
            st = rast.forward(cam, **inputs, sh_degree=D, max_rendered=cap)
            return st, rast.backward(st, dpix), None

    # Warm-up: the W steps asked for, and at least WARMUP_FLOOR_S seconds of steps, so that the
    # timed steps see the GPU at its steady clocks (a fresh box's first process measured ~3.5 %
    # slower with 5 warm-up steps than the next process, profiles/r03_experiments/bench_warm.jsonl).
    # The timed region below is unchanged: exactly K full steps.
    tw0, warm_steps = time.perf_counter(), 0
    # (one rank only: ranks step in lockstep through collectives, so their counts must match)
    while warm_steps < args.warmup or (dist is None and time.perf_counter() - tw0 < WARMUP_FLOOR_S):
        step()
        warm_steps += 1
        if warm_steps >= args.warmup:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    warm_s = time.perf_counter() - tw0
    # Stage breakdown: a separate, untimed pass with HIP events around every stage (each
    # event pair adds ~10 us of dispatch gap, so the timed loop below carries only the
    # dominant kernel's pair -- its live duration feeds `roofline`).
    stages, dom_stage = {}, None
    if not args.no_stage_events:
        if dist:
            dist.barrier()
        native.profile_enable()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        stages = native.profile_read()
        native.profile_enable(0)
        cand = {k: v for k, v in stages.items() if v[1] and k in ALG_STAGES}
        dom_stage = max(cand, key=lambda k: cand[k][0]) if cand else None
    if dist:
        dist.barrier()
    if dom_stage is not None:
        native.profile_enable(1 << native.STAGES.index(dom_stage))
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        st, g, sh = step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    live = native.profile_read() if dom_stage is not None else {}
    native.profile_enable(0)
    if world > 1:
        plan.check()  # the last `lag` steps' agreed overflow checks, before any count is reported
    if dist:
        tt = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    ms_per_step = 1e3 * elapsed / args.steps
    value = args.steps / elapsed  # whole-image forward+backward iterations per second (job)

    K = st.num_rendered  # raises on a binning overflow
    tiles = gx * gy
    M = (D + 1) ** 2
    if world > 1:  # K, pixels and tiles of the band; P and V of the shard
        V = int((sh.radii > 0).sum())
        P_local = plan.g1 - plan.g0
        pix_local = (min(band[1] * 16, H) - band[0] * 16) * W
        tiles_local = (band[1] - band[0]) * gx
    else:
        V = int((st.radii > 0).sum())
        P_local, pix_local, tiles_local = P, W * H, tiles
    alg = algorithmic_bytes(P_local, V, K, pix_local, tiles_local, M)
    result = {
        "metric": config_metric(args.config),
        "value": round(value, 3), "unit": "iters/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "warmup_run": {"steps": warm_steps, "s": round(warm_s, 3)},
        "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": f"{args.config}: {P} Gaussians, {W}x{H}, SH degree {D}, fwd+bwd",
                   "gaussians": P, "width": W, "height": H, "sh_degree": D,
                   "parallelism": (f"Gaussian shards x instance-balanced tile-row bands x{world}" if world > 1
                                   else "single GPU")},
        "mpixel_per_s": round(W * H * value / 1e6, 2),
        "counts": {"visible": V, "num_rendered": K, "tiles": tiles},
    }
    if world > 1:
        result["exchange"] = {"impl": (plan.impl if isinstance(plan, CppShard) else
                                       f"bands.ShardStep over torch.distributed ({args.dist_backend})"),
                              "backend": args.dist_backend,
                              "band_rows": plan.rows, "pair_cap": plan.pair_cap, "band_capacity": plan.capacity,
                              "band_instances": plan.band_instances, "counts_are": "rank 0's shard / band",
                              "comm_world": (plan.comm_world if isinstance(plan, CppShard) else dist.get_world_size()),
                              "overflow_checked": "every step, agreed across ranks"}
        if result["exchange"]["comm_world"] != world:
            raise SystemExit(f"communicator counts {result['exchange']['comm_world']} ranks, WORLD_SIZE {world}")
    if stages and rank == 0 and dom_stage in live and live[dom_stage][1]:
        result["stage_ms"] = {k: round(ms / args.steps, 4) for k, (ms, n) in stages.items() if n}
        # every stage's algorithmic bytes over its measured time, as a fraction of 8 TB/s (tracked
        # per round: VERDICT r04 item 5); the blend stages are bound by VALU issue, not HBM
        sb = stage_bytes(P_local, V, K, pix_local, tiles_local, M)
        if "duplicate" not in result["stage_ms"] and "tile_sort" in result["stage_ms"]:
            # row-bucketed binning (gsr_sort.hip): F3, the tile sort and F5 are one timed stage
            sb["tile_sort"] += sb["duplicate"] + sb["finalize"]
            result["binning"] = "row-bucketed: F3 + tile sort + F5 timed as tile_sort"
        result["stage_hbm_frac"] = {k: round(sb[k] / (result["stage_ms"][k] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                                    for k in sb if result["stage_ms"].get(k)}
        dom = dom_stage
        launches_per_step = max(live[dom][1] // args.steps, 1)
        mean_ms = live[dom][0] / live[dom][1]  # HIP events in the timed loop, launch stream
        bytes_launch = alg[dom] / launches_per_step
        achieved = bytes_launch / (mean_ms * 1e-3) / 1e9
        kernel_name = {"blend_fwd": "blend_forward_kernel", "blend_bwd": "blend_backward_kernel",
                       "preprocess": "preprocess_kernel", "preprocess_bwd": "preprocess_backward_kernel"}.get(dom, dom)
        pmc = pmc_record(kernel_name, args.config)
        # The contract's fields (bound / achieved / peak / unit / frac / traffic) are all the HBM
        # roofline of the dominant kernel, consistently.  The blend loops issue VALU work per
        # (pixel, record) pair and reuse LDS-staged records 256x per tile, so the roofline that
        # BINDS them is VALU issue: `binding` names it and `valu_issue` carries its
        # own achieved / peak / frac.
        binding = "valu_issue" if dom in ("blend_fwd", "blend_bwd") else "hbm"
        result["roofline"] = {"bound": "hbm", "binding": binding, "kernel": kernel_name,
                              "achieved": round(achieved, 2),
                              "lib_stamp": (lib_stamp() or "")[:16],
                              "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                              # PMC passes are of the N = 1 launch; a band launch has no committed counts
                              "traffic": pmc.get("hbm_bytes_per_launch") if world == 1 else None, "mean_launch_ms": round(mean_ms, 4),
                              "algorithmic_bytes_per_launch": int(bytes_launch)}
        if "write_size_kib" in pmc and world == 1:
            # B1's partial-entry writes against the algorithmic 36 B per visible Gaussian (VERDICT r05
            # item 5): the per-(tile, instance) partials the deterministic hand-off costs
            wb = pmc["write_size_kib"] * 1024
            result["roofline"]["write_bytes_per_launch"] = int(wb)
            if dom == "blend_bwd":
                result["roofline"]["write_over_algorithmic"] = round(wb / (V * 36), 3) if V else None
        if "valu_insts_per_launch" in pmc and world == 1:  # PMC counts are of the N = 1 launch
            # F6/B1 are bound by VALU issue, not HBM: the kernel's measured
            # instruction count over its measured duration, against the spec issue peak (1024
            # SIMDs x one wave64 op per 2 cycles at 2.4 GHz).
            slots = VALU_ISSUE_PER_S * mean_ms * 1e-3
            result["roofline"]["valu_issue"] = {
                "insts_per_launch": pmc["valu_insts_per_launch"],
                "achieved": round(pmc["valu_insts_per_launch"] / (mean_ms * 1e-3), 1),
                "peak": VALU_ISSUE_PER_S, "unit": "wave64 VALU insts/s",
                "frac": round(pmc["valu_insts_per_launch"] / slots, 4)}
        total_alg = sum(alg.values())
        result["pipeline_roofline"] = {
            "algorithmic_bytes_per_step": int(total_alg),
            "achieved_GBs": round(total_alg / (ms_per_step * 1e-3) / 1e9, 2),
            "frac_of_8TBs": round(total_alg / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import gsr_oracle  # cpu_baseline leg only: the checker / reported baseline
        cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
        os.environ.setdefault("OMP_NUM_THREADS", str(cores))
        times, f, gc = [], None, None
        for it in range(4):  # one warm-up, then the median of three
            c0 = time.perf_counter()
            f = gsr_oracle.forward(cam, scene.means3D, scene.opacities, scene.scales, scene.rotations,
                                   scene.sh_dc, scene.sh_rest, sh_degree=D)
            gc = f.state.backward(dpix_np)
            if it:
                times.append(time.perf_counter() - c0)
        cpu_s = float(np.median(times))
        col = st.color.cpu().numpy().astype(np.float64)
        mse = float(np.mean((col - f.color) ** 2))
        rel = {}
        for k in ("means3D", "opacities", "scales", "rotations", "sh_dc", "sh_rest"):
            a = g[k].cpu().numpy().reshape(gc[k].shape).astype(np.float64)
            rel[k] = float(np.linalg.norm(a - gc[k]) / max(np.linalg.norm(gc[k]), 1e-30))
        result["cpu_baseline"] = {"value": round(1.0 / cpu_s, 5), "unit": "iters/s", "cores": cores,
                                  "kind": "port", "sample": f"full {args.config} forward+backward on the CPU "
                                  f"oracle, median of 3 after 1 warm-up ({', '.join(f'{x:.2f}' for x in times)} s; "
                                  f"OpenMP {cores} threads)",
                                  "cpu_model": cpu_model(), "nproc": os.cpu_count(),
                                  "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
                                  # the GPU box grants this job OMP_NUM_THREADS host threads (the
                                  # harness sets 16 per GPU and forbids raising it); nproc counts
                                  # the whole machine.  A whole-machine figure is an estimate,
                                  # linear in threads (an upper bound for the CPU):
                                  "full_machine_linear_estimate": round(os.cpu_count() / cores / cpu_s, 4)}
        if "roofline" in result:
            work = f.state.blend_work()
            floor_insts = (work["f6_wave_visits"] * F6_VISIT_VALU + work["b1_stripe_evals"] * B1_STRIPE_VALU +
                           work["b1_contrib_evals"] * B1_CONTRIB_VALU)
            floor_ms = floor_insts / VALU_ISSUE_PER_S * 1e3
            meas = sum(result.get("stage_ms", {}).get(k, 0.0) for k in ("blend_fwd", "blend_bwd"))
            vb = {"pairs": f.state.forward_pairs(), "work": work,
                  "body_valu": {"f6_per_wave_visit": F6_VISIT_VALU, "b1_per_stripe_eval": B1_STRIPE_VALU,
                                "b1_contribution": B1_CONTRIB_VALU},
                  "source": "ISA loop bodies (DESIGN §6) x oracle-counted culled evaluations (lower bounds)",
                  "floor_insts": int(floor_insts), "peak_insts_per_s": VALU_ISSUE_PER_S,
                  "floor_ms_f6_b1": round(floor_ms, 4), "measured_ms_f6_b1": round(meas, 4),
                  "frac": round(floor_ms / meas, 4) if meas else None}
            f6, b1 = pmc_record("blend_forward_kernel", args.config), pmc_record("blend_backward_kernel", args.config)
            if "valu_insts_per_launch" in f6 and "valu_insts_per_launch" in b1:
                # the instructions the kernels issue beyond the floor bodies (set-up, loads,
                # reductions, loop control): this build's PMC counts
                issued = f6["valu_insts_per_launch"] + b1["valu_insts_per_launch"]
                vb["pmc_valu_insts_f6_b1"] = issued
                vb["overhead_share_of_issued"] = round(1.0 - floor_insts / issued, 4)
            result["roofline"]["valu_pair_bound"] = vb
        result["parity"] = {"psnr_db_vs_cpu": round(10 * math.log10(1.0 / mse), 2) if mse > 0 else float("inf"),
                            "rgb_rel_l2": float(np.linalg.norm(col - f.color) / np.linalg.norm(f.color)),
                            "grad_rel_l2_max": max(rel.values()),
                            "num_rendered_equal": int(f.num_rendered) == K}
    if rank == 0:
        print(json.dumps(result))
    if dist:
        dist.destroy_process_group()


def train_main(args):
    """One training iteration per step (trainer.GaussianTrainer.step, densification off so the
    Gaussian count stays fixed): N = 1 only.  Stage times from torch events on the launch
    stream (the C-ABI calls run on torch's current stream); roofline for the fused Adam, the
    only new HBM-bound stream whose bytes scale with P x 59 floats."""
    Tr = importlib.import_module(f"{PKG}.trainer")
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        raise SystemExit("--mode train runs on one GPU")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = CONFIGS[args.config]
    P, W, H, D = cfg["P"], cfg["W"], cfg["H"], cfg["D"]
    cam = gr.synthetic_camera(W, H)
    scene = sc.make_scene(cam, P, max_sh_degree=max(D, 0), seed=0)
    tr = Tr.GaussianTrainer(scene.means3D, scene.sh_dc, scene.sh_rest, scene.raw_opacities, scene.raw_scales,
                            scene.raw_rotations, max_sh_degree=D, device=dev)
    tr.active_sh_degree = D
    gt = torch.tensor(sc.make_dL_dpix(cam, seed=2), device=dev) * 0.5 + 0.5  # synthetic target in [0, 1]
    it = [1]

    def step():
        out = tr.step(it[0], cam, gt, densify=False)
        it[0] += 1
        return out

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # stage split (separate pass): events between the phases of one iteration
    ev = lambda: torch.cuda.Event(enable_timing=True)
    names = ("activate+render", "loss", "backward", "stats+adam")
    acc = dict.fromkeys(names, 0.0)
    adam_ms = 0.0
    for _ in range(args.steps):
        e = [ev() for _ in range(6)]
        e[0].record()
        st = tr.render(cam)
        e[1].record()
        stats, maps = tr.k.loss_forward(st.color, gt, tr.opt.lambda_dssim)
        dimg = tr.k.loss_backward(st.color, gt, tr.opt.lambda_dssim, maps)
        e[2].record()
        g = tr.rast.backward(st, dimg)
        e[3].record()
        tr.k.densify_stats(st.radii, g["means2D"], tr.max_radii2D, tr.xyz_gradient_accum, tr.denom)
        grads = {"xyz": g["means3D"], "f_dc": g["sh_dc"], "f_rest": g["sh_rest"], "opacity": g["opacities"],
                 "scaling": g["scales"], "rotation": g["rotations"]}
        e[4].record()
        tr.optimizer_step(grads)
        e[5].record()
        torch.cuda.synchronize()
        for i, n in enumerate(names[:3]):
            acc[n] += e[i].elapsed_time(e[i + 1])
        acc["stats+adam"] += e[3].elapsed_time(e[5])
        adam_ms += e[4].elapsed_time(e[5])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    ms = 1e3 * elapsed / args.steps
    floats = sum(v.numel() for v in tr.params.values())
    adam_bytes = floats * 28  # p, m, v read + written, grad read (f32)
    adam_mean = adam_ms / args.steps
    stats = out["stats"].cpu().tolist()
    res = {"metric": f"training iterations/s at {config_label(args.config)} (activations + render + L1/D-SSIM "
                     "loss + backward + densification statistics + fused Adam)",
           "value": round(args.steps / elapsed, 3), "unit": "iters/s", "n_gpus": 1, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "strong",
           "vs_baseline": None, "dtype": "f32", "data": "synthetic",
           "config": {"workload": f"{args.config} training step: {P} Gaussians, {W}x{H}, SH degree {D}, "
                                  f"densification off", "gaussians": P, "width": W, "height": H, "sh_degree": D},
           "stage_ms": {k: round(v / args.steps, 4) for k, v in acc.items()},
           "roofline": {"bound": "hbm", "kernel": "adam_kernel", "achieved": round(adam_bytes / (adam_mean * 1e-3) / 1e9, 2),
                        "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(adam_bytes / (adam_mean * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "traffic": None,
                        "mean_launch_ms": round(adam_mean, 4), "algorithmic_bytes_per_launch": adam_bytes,
                        "note": "activation backward fused; the event pair brackets the single adam launch"},
           "loss": {"loss": stats[0], "l1": stats[1], "ssim": stats[2]}}
    print(json.dumps(res))


def views_main(args):
    """V cameras around the scene per step, forward + backward of each view.
    Batched (gsr_forward_batch: one host wait per batch) against the same views one
    gsr_forward at a time; value = batched views/s.  N = 1 only."""
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        raise SystemExit("--mode views runs on one GPU")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = CONFIGS[args.config]
    P, W, H, D = cfg["P"], cfg["W"], cfg["H"], cfg["D"]
    cam0 = gr.synthetic_camera(W, H)
    scene = sc.make_scene(cam0, P, max_sh_degree=max(D, 0), seed=0)
    fx = math.radians(60.0)
    fy = 2 * math.atan(math.tan(fx / 2) * H / W)
    cams = []
    for v in range(args.views):  # small yaw sweep around the synthetic camera
        a = math.radians(-10.0 + 20.0 * v / max(args.views - 1, 1))
        Rm = np.array([[math.cos(a), 0, math.sin(a)], [0, 1, 0], [-math.sin(a), 0, math.cos(a)]])
        cams.append(gr.make_camera(Rm, np.zeros(3), fx, fy, W, H))
    rast = R.CAbiRasterizer(dev)
    t = lambda a: torch.tensor(a, device=dev)
    inputs = dict(means3D=t(scene.means3D), opacities=t(scene.opacities), scales=t(scene.scales),
                  rotations=t(scene.rotations), sh_dc=t(scene.sh_dc), sh_rest=t(scene.sh_rest))
    dpix = t(sc.make_dL_dpix(cam0, seed=1))

    def batched():
        for st in rast.forward_batch(cams, **inputs, sh_degree=D):
            rast.backward(st, dpix)

    nat = R.native
    passes = [cams[i:i + nat.GSR_MAX_VIEWS] for i in range(0, len(cams), nat.GSR_MAX_VIEWS)]
    dpix_v = {len(p): dpix.expand(len(p), *dpix.shape).contiguous() for p in passes}

    def one_pass():  # gsr_forward_views / gsr_backward_views: one launch per stage per <= 8 views
        for p in passes:
            rast.backward_views(rast.forward_views(p, **inputs, sh_degree=D), dpix_v[len(p)])

    def single():
        for c in cams:
            rast.backward(rast.forward(c, **inputs, sh_degree=D), dpix)

    res = {}
    for name, fn in (("single", single), ("batched", batched), ("views", one_pass)) * 2:
        for _ in range(args.warmup):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            fn()
        torch.cuda.synchronize()
        res.setdefault(name, []).append(args.steps * args.views / (time.perf_counter() - t0))
    v1, b, s1 = max(res["views"]), max(res["batched"]), max(res["single"])
    print(json.dumps({
        "metric": f"forward+backward views/s, {args.views} cameras per step", "value": round(v1, 2),
        "unit": "views/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(1e3 * args.views / v1, 4), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": f"{args.config} x {args.views} views (yaw -10..10 deg), gsr_forward_views + "
                               f"gsr_backward_views (one pass per <= {nat.GSR_MAX_VIEWS} views)", "gaussians": P,
                   "width": W, "height": H, "sh_degree": D},
        "single_view_calls_views_per_s": round(s1, 2), "batch_views_per_s": round(b, 2),
        "views_speedup": round(v1 / s1, 4), "batch_speedup": round(b / s1, 4)}))


def loop_main(args):
    """BASELINE configs[4]: the full training loop (train_loop.train, train_utils.cpp:128-145 order,
    params.h:50-91 defaults) on a synthetic Mip-NeRF360-scale scene: --views cameras on an orbit,
    ground truth rendered from a --loop-gt Gaussian cloud, training from a --loop-init point
    cloud.  value = training iterations/s over the whole run (densification included)."""
    L = importlib.import_module(f"{PKG}.train_loop")
    T = importlib.import_module(f"{PKG}.trainer")
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        raise SystemExit("--mode loop runs on one GPU")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    W, H = (int(v) for v in args.loop_size.split("x"))
    t0 = time.perf_counter()
    scene = L.synthetic_scene(args.loop_gt, args.loop_init, args.loop_views, W, H, seed=0, device=dev,
                              texture=args.loop_texture, gt_scale=args.loop_gt_scale)
    setup_s = time.perf_counter() - t0
    opt = T.OptimizationParams(iterations=args.iters)
    if args.loop_engine == "cpp":
        res = _loop_cpp(L, scene, opt, args)
    else:
        res = L.train(scene, opt=opt, max_sh_degree=3, log_every=500, device=dev, progress_every=1000)
    print(json.dumps({
        "metric": "training iterations/s, full train.cpp loop (render + L1/D-SSIM + backward + densification + Adam)",
        "value": round(res.iters_per_s, 3), "unit": "iters/s", "n_gpus": 1, "steps": res.iterations, "warmup": 0,
        "ms_per_step": round(1e3 * res.seconds / res.iterations, 4), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": f"configs[4]: {args.iters} iterations, {args.loop_views} views {W}x{H}, ground truth "
                               f"{args.loop_gt} Gaussians (texture {args.loop_texture}, scale {args.loop_gt_scale}), init "
                               f"{args.loop_init} points, "
                               f"SH 3", "width": W, "height": H, "views": args.loop_views,
                   "engine": ("C++ loop tests/cpp/train_main.cpp over gsr::Trainer" if args.loop_engine == "cpp"
                              else "Python train_loop.train over trainer.GaussianTrainer")},
        "seconds": round(res.seconds, 2), "setup_seconds": round(setup_s, 2),
        "final_gaussians": res.final_points, "peak_gaussians": res.peak_points,
        "binning_overflows": res.binning_overflows, "exact_k_reads": res.exact_k_reads,
        "gaussians_after_densify": res.num_points[::10] + res.num_points[-1:],
        "loss_curve": [(i, round(l, 5)) for i, l, _, _ in res.loss][::4] + [(res.loss[-1][0], round(res.loss[-1][1], 5))]}))


def _loop_cpp(L, scene, opt, args):
    """Run the C++ loop executable on `scene` (written to a GSRLOOP1 file); returns a LoopResult."""
    import subprocess
    import tempfile
    exe = os.path.join(ROOT, PKG, "lib", "gsr_train_loop")
    if not os.path.exists(exe):
        raise SystemExit(f"{exe} missing: run __graft_entry__.build()")
    with tempfile.TemporaryDirectory() as d:
        fin, fres = os.path.join(d, "scene.bin"), os.path.join(d, "res.json")
        L.write_scene(fin, scene, args.iters, opt, max_sh_degree=3, log_every=500, progress_every=1000)
        r = subprocess.run([exe, fin, fres], stdout=subprocess.PIPE, text=True)
        if r.returncode != 0:
            raise SystemExit(f"gsr_train_loop failed ({r.returncode}): {r.stdout}")
        j = json.load(open(fres))
    return L.LoopResult(iterations=j["iterations"], seconds=j["seconds"], iters_per_s=j["iters_per_s"],
                        num_points=[tuple(x) for x in j["num_points"]], loss=[tuple(x) for x in j["loss"]],
                        final_points=j["final_points"], peak_points=j["peak_points"],
                        binning_overflows=j["binning_overflows"], exact_k_reads=j["exact_k_reads"])


if __name__ == "__main__":
    main()
