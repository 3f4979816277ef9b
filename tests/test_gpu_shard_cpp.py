"""GPU: the C++ multi-GPU step (gsr::ShardStep, csrc/torch/gsr_shard.h) -- the native twin of
bands.ShardStep, so that a C++ src/train.cpp runs the sharded path (north_star: host code stays
C++).  Every case runs the executable lib/gsr_shard_step (tests/cpp/shard_main.cpp), one process
per rank, and compares with the single-GPU CAbiRasterizer on the same scene:

* two processes on the box's one GPU over the host-staged c10d::Store exchange (RCCL refuses two
  ranks on one device): gathered image and radii bit-exact, leaf gradients within 1e-5 rel-L2
  (band-order sums vs emission-order sums), as tests/test_gpu_multiproc.py bars the Python path;
* a forced pair_cap below the true splat counts: BOTH ranks raise ShardOverflowError for step 0
  at the same call (the status words ride in the image all-gather, so every rank checks every
  rank's counts, `lag` steps later);
* one rank over RCCL itself (gsr_comm_*, a world-1 communicator), eager and captured into a
  hipGraph (replayed from the second step): both equal the single-GPU render, and each other bit
  for bit;
* the same through the Python binding (the benchmark's multi-GPU path).
"""
import os
import re
import socket
import subprocess
import tempfile

import numpy as np
import pytest
import torch

from conftest import ROOT, pkg, rel_l2

pytestmark = pytest.mark.gpu
EXE = os.path.join(ROOT, "3d_gaussian_splatting_amd", "lib", "gsr_shard_step")
W, H, P = 640, 480, 40000
GRADS = [("means2D", 3), ("opacities", 1), ("means3D", 3), ("sh_dc", 3), ("sh_rest", 45), ("scales", 3),
         ("rotations", 4)]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def scene():
    gr, sc = pkg("graphics"), pkg("scene")
    cam = gr.synthetic_camera(W, H)
    s = sc.make_scene(cam, P, max_sh_degree=3, seed=61)
    dpix = sc.make_dL_dpix(cam, seed=62)
    return cam, s, dpix


@pytest.fixture(scope="module")
def reference(scene):
    cam, s, dpix = scene
    rast = pkg("rasterizer").CAbiRasterizer("cuda")
    args = (cam, s.means3D, s.opacities, s.scales, s.rotations, s.sh_dc, s.sh_rest)
    full = rast.forward(*args, sh_degree=3)
    g = rast.backward(full, dpix)
    return full.color.cpu().numpy(), full.radii.cpu().numpy(), {k: v.cpu().numpy() for k, v in g.items()}


def _write_scene(path, cam, s, dpix):
    M = s.sh_rest.reshape(P, -1, 3).shape[1]
    with open(path, "wb") as f:
        f.write(b"GSRSHRD1")
        f.write(np.array([P, W, H, 3, M], np.int32).tobytes())
        f.write(np.concatenate([[cam.tanfovx, cam.tanfovy], np.asarray(cam.viewmatrix, np.float32).ravel(),
                                np.asarray(cam.projmatrix, np.float32).ravel(),
                                np.asarray(cam.campos, np.float32).ravel()]).astype(np.float32).tobytes())
        for a in (s.means3D, s.opacities, s.scales, s.rotations, s.sh_dc, s.sh_rest, dpix):
            f.write(np.ascontiguousarray(a, np.float32).tobytes())


def _read_out(path, world):
    b = open(path, "rb").read()
    assert b[:8] == b"GSRSHOUT"
    o = 8
    hdr = np.frombuffer(b, np.int64, 8, o)
    o += 64
    g0, g1, pair_cap, capacity, done, ovf_step, ovf_rank, graph = (int(v) for v in hdr)
    rows = np.frombuffer(b, np.int32, world + 1, o)
    o += 4 * (world + 1)
    out = dict(g0=g0, g1=g1, pair_cap=pair_cap, capacity=capacity, done=done, ovf_step=ovf_step,
               ovf_rank=ovf_rank, graph=graph, rows=rows)
    if done:
        n = g1 - g0
        out["image"] = np.frombuffer(b, np.float32, 3 * H * W, o).reshape(3, H, W)
        o += 12 * H * W
        out["radii"] = np.frombuffer(b, np.int32, n, o)
        o += 4 * n
        for k, c in GRADS:
            out[k] = np.frombuffer(b, np.float32, n * c, o).reshape(n, c)
            o += 4 * n * c
        rest = (len(b) - o) // 4
        assert rest % (3 * H * W) == 0
        out["images"] = np.frombuffer(b, np.float32, rest, o).reshape(-1, 3, H, W)  # GSR_ALL_IMAGES
    return out


def _run(scene_path, world, transport, d, extra=None, graph=False, steps=2):
    assert os.path.exists(EXE), "run __graft_entry__.build()"
    port = str(_free_port())
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=port,
                   GSR_TRANSPORT=transport, GSR_GRAPH="1" if graph else "0", GSR_STEPS=str(steps), **(extra or {}))
        procs.append(subprocess.Popen([EXE, scene_path, os.path.join(d, f"out{r}.bin")], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    logs = []
    for p in procs:
        try:
            logs.append(p.communicate(timeout=150)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            pytest.fail("gsr_shard_step timed out")
    for p, log in zip(procs, logs):
        assert p.returncode == 0, log
    print("\n".join(logs))
    outs = [_read_out(os.path.join(d, f"out{r}.bin"), world) for r in range(world)]
    for o, log in zip(outs, logs):
        o["log"] = log
    return outs


def _check_against(outs, reference, world):
    img, radii, g = reference
    for o in outs:
        np.testing.assert_array_equal(o["image"], img)
    np.testing.assert_array_equal(np.concatenate([o["radii"] for o in outs]), radii)
    for k, c in GRADS:
        a = np.concatenate([o[k] for o in outs])
        ref = g[k].reshape(P, -1)[:, :c]
        assert rel_l2(a, ref) <= 1e-5, k


def test_two_processes_store_exchange(scene, reference):
    cam, s, dpix = scene
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "scene.bin")
        _write_scene(path, cam, s, dpix)
        outs = _run(path, 2, "store", d, steps=6)
    assert all(o["done"] == 6 and o["ovf_step"] == -1 for o in outs)
    # the host-staged exchange deletes its payload and barrier keys (the last rank out
    # of each barrier does): six steps leave no per-step keys in the store (before: >= 12)
    keys = [int(m) for m in re.findall(r"store_keys (\d+)", outs[0]["log"])]
    assert keys and max(keys) <= 6, outs[0]["log"]
    assert outs[0]["rows"][1] not in (0, cam.grid[1])  # a real two-band split
    assert [o["g0"] for o in outs] == [0, outs[0]["g1"]] and outs[1]["g1"] == P
    _check_against(outs, reference, 2)


def test_two_processes_overflow_agreed(scene):
    cam, s, dpix = scene
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "scene.bin")
        _write_scene(path, cam, s, dpix)
        outs = _run(path, 2, "store", d, extra={"GSR_FORCE_PAIR_CAP": "64"}, steps=4)
    # step 0 overflowed on some rank; both ranks raise for it at the same call (step 2, lag 2)
    for o in outs:
        assert o["ovf_step"] == 0 and o["done"] == 2, o
    assert outs[0]["ovf_rank"] == outs[1]["ovf_rank"]


def test_rccl_world1_eager_and_graph(scene, reference):
    cam, s, dpix = scene
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "scene.bin")
        _write_scene(path, cam, s, dpix)
        eager = _run(path, 1, "rccl", d, steps=2)
        graph = _run(path, 1, "rccl", d, graph=True, steps=3)
    assert eager[0]["graph"] == 0 and graph[0]["graph"] == 1 and graph[0]["done"] == 3
    _check_against(eager, reference, 1)
    for k in ["image", "radii"] + [k for k, _ in GRADS]:
        np.testing.assert_array_equal(graph[0][k], eager[0][k], err_msg=k)


def test_python_binding_rccl_graph(scene, reference):
    """The benchmark's path: ext.ShardStep over ext.rccl_exchange, graph replay."""
    cam, s, dpix = scene
    ext = pkg("native").load_torch_ext()
    R = pkg("rasterizer")
    dev = torch.device("cuda", 0)
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a, np.float32), device=dev)
    inputs = dict(means3D=t(s.means3D), opacities=t(s.opacities), scales=t(s.scales), rotations=t(s.rotations),
                  sh_dc=t(s.sh_dc).reshape(P, 1, 3), sh_rest=t(s.sh_rest).reshape(P, -1, 3))
    ex = ext.rccl_exchange(ext.rccl_unique_id(), 0, 1)
    st = ext.ShardStep(ex, R.ext_camera(cam), inputs, 3, graph=True)
    st.plan()
    d = t(dpix)
    outs = [st.step(d) for _ in range(3)]
    st.check()
    assert st.graph_active
    img, grads, radii = outs[-1]
    ref_img, ref_radii, g = reference
    np.testing.assert_array_equal(img.cpu().numpy(), ref_img)
    np.testing.assert_array_equal(radii.cpu().numpy(), ref_radii)
    for k, c in GRADS:
        assert rel_l2(grads[k].cpu().numpy().reshape(P, -1)[:, :c], g[k].reshape(P, -1)[:, :c]) <= 1e-5, k


def test_python_binding_camera_move_rebalances(scene):
    """A moving camera through the C++ step: set_camera drops the captured graph, and with
    rebalance_every = 1 the next step re-plans for the new view first; its image and radii equal
    the single-GPU render of that view, and later steps replay a graph captured for it."""
    import math
    cam, s, dpix = scene
    ext = pkg("native").load_torch_ext()
    R, gr = pkg("rasterizer"), pkg("graphics")
    dev = torch.device("cuda", 0)
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a, np.float32), device=dev)
    inputs = dict(means3D=t(s.means3D), opacities=t(s.opacities), scales=t(s.scales), rotations=t(s.rotations),
                  sh_dc=t(s.sh_dc).reshape(P, 1, 3), sh_rest=t(s.sh_rest).reshape(P, -1, 3))
    ex = ext.rccl_exchange(ext.rccl_unique_id(), 0, 1)
    st = ext.ShardStep(ex, R.ext_camera(cam), inputs, 3, graph=True)
    st.plan()
    d = t(dpix)
    for _ in range(2):
        st.step(d)
    assert st.graph_active
    cam_b = gr.make_camera(np.eye(3), np.array([0.0, 0.8, 0.0]), 2 * math.atan(cam.tanfovx),
                           2 * math.atan(cam.tanfovy), cam.width, cam.height)
    st.set_camera(R.ext_camera(cam_b))
    assert not st.graph_active
    st.set_rebalance_every(1)
    img, _, radii = st.step(d)
    assert st.replans == 1
    full = R.CAbiRasterizer(dev).forward(cam_b, **inputs, sh_degree=3)
    np.testing.assert_array_equal(img.cpu().numpy(), full.color.cpu().numpy())
    np.testing.assert_array_equal(radii.cpu().numpy(), full.radii.cpu().numpy())
    st.set_rebalance_every(0)
    img2, _, _ = st.step(d)
    img3, _, _ = st.step(d)
    st.check()
    assert st.graph_active
    np.testing.assert_array_equal(img3.cpu().numpy(), full.color.cpu().numpy())


def test_python_binding_overflow_guard_skips_adam(scene):
    """the C++ step's agreed overflow word is on the device after every step
    (0 for a step within the plan's capacities, the number of overflowing ranks otherwise), and a
    fused Adam step guarded by it (gsr_adam_step_guarded, guard_cap 0) leaves the parameters
    untouched for the truncated step -- before the lagged host check raises."""
    cam, s, dpix = scene
    ext = pkg("native").load_torch_ext()
    R, T = pkg("rasterizer"), pkg("trainer")
    dev = torch.device("cuda", 0)
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a, np.float32), device=dev)
    inputs = dict(means3D=t(s.means3D), opacities=t(s.opacities), scales=t(s.scales), rotations=t(s.rotations),
                  sh_dc=t(s.sh_dc).reshape(P, 1, 3), sh_rest=t(s.sh_rest).reshape(P, -1, 3))
    ex = ext.rccl_exchange(ext.rccl_unique_id(), 0, 1)
    assert ex.comm_world == 1
    st = ext.ShardStep(ex, R.ext_camera(cam), inputs, 3, graph=True)
    st.plan()
    assert st.exchange_world == 1 and st.exchange_name == "rccl"
    d = t(dpix)
    k = T.TrainKernels(dev)

    def adam(grads):
        p = inputs["means3D"].clone()
        m, v = torch.zeros_like(p), torch.zeros_like(p)
        k.adam_step([dict(param=p, grad=grads["means3D"].contiguous(), exp_avg=m, exp_avg_sq=v, act=0, step=1,
                          lr=1e-3)], guard=(st.overflow_guard, 0))
        torch.cuda.synchronize()
        return p

    _, g, _ = st.step(d)
    assert int(st.overflow_guard.item()) == 0
    assert not torch.equal(adam(g), inputs["means3D"])  # applied
    st.set_pair_cap(64)  # far below the true splat counts: the step is truncated
    _, g, _ = st.step(d)
    assert int(st.overflow_guard.item()) == 1
    assert torch.equal(adam(g), inputs["means3D"])  # skipped on the device
    with pytest.raises(OverflowError):
        st.check()


def _cam_path(cam, n):
    """A moving camera: yaw -6..6 degrees with the view sliding 0.9 down -- the scene's instances
    move up the image and the balanced cuts must follow."""
    import math
    gr = pkg("graphics")
    fx, fy = 2 * math.atan(cam.tanfovx), 2 * math.atan(cam.tanfovy)
    out = []
    for i in range(n):
        a = math.radians(-6.0 + 12.0 * i / (n - 1))
        Rm = np.array([[math.cos(a), 0, math.sin(a)], [0, 1, 0], [-math.sin(a), 0, math.cos(a)]])
        out.append(gr.make_camera(Rm, np.array([0.0, 0.9 * i / (n - 1), 0.0]), fx, fy, cam.width, cam.height))
    return out


def test_two_processes_live_replan_camera_path(scene):
    """the C++ step re-cuts its bands from the statistics every step carries
    (GSR_FLAG_ROW_SPANS rows in the status footer; no probe, no extra collective), here over a
    24-pose camera path through the host-staged exchange in two processes: no overflow, cuts that
    move with the view, and every step's gathered image equal to the single-GPU render of its
    camera bit for bit.  Per-step wall times (synchronised) go to gpurun_out/ for the re-plan
    cost (profiles/r05_live_replan_*)."""
    cam, s, dpix = scene
    path_cams = _cam_path(cam, 24)
    rast = pkg("rasterizer").CAbiRasterizer("cuda")
    args = (s.means3D, s.opacities, s.scales, s.rotations, s.sh_dc, s.sh_rest)
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "scene.bin")
        _write_scene(path, cam, s, dpix)
        cp = os.path.join(d, "cams.bin")
        with open(cp, "wb") as f:
            for c in path_cams:
                f.write(np.concatenate([[c.tanfovx, c.tanfovy], np.asarray(c.viewmatrix, np.float32).ravel(),
                                        np.asarray(c.projmatrix, np.float32).ravel(),
                                        np.asarray(c.campos, np.float32).ravel()]).astype(np.float32).tobytes())
        outs = _run(path, 2, "store", d, steps=24,
                    extra={"GSR_CAM_PATH": cp, "GSR_LIVE": "1", "GSR_ALL_IMAGES": "1", "GSR_TIMING": "1"})
    for o in outs:
        assert o["done"] == 24 and o["ovf_step"] == -1, o["log"]
        assert o["images"].shape[0] == 24
    replans = [int(m) for m in re.findall(r"live_replans (\d+)", outs[0]["log"])]
    assert replans and replans[0] >= 2, outs[0]["log"]  # the cuts followed the view
    for i, c in enumerate(path_cams):
        want = rast.forward(c, *args, sh_degree=3).color.cpu().numpy()
        for o in outs:
            np.testing.assert_array_equal(o["images"][i], want, err_msg=f"step {i}")
    timing = [ln for o in outs for ln in o["log"].splitlines() if ln.startswith('{"rank"')]
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "live_replan_timing.jsonl"), "w") as f:
        f.write("\n".join(timing) + "\n")
