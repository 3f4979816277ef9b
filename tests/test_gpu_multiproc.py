"""GPU: the multi-GPU step (bands.ShardStep over the HIP gsr_shard_* / gsr_band_* calls) in TWO
real processes -- torch.multiprocessing spawn, a gloo process group, both ranks on the box's one
GPU (the N-GPU runs are the driver's).  Every byte of the exchange crosses a process boundary:
the splat all-to-all, the band-image all-gather and the gradient all-to-all.

Checks: the gathered image equals the single-process CAbiRasterizer render bit for
bit, the radii too, and the leaf gradients gathered from both shards match within 1e-5
relative L2 (band-order sums vs the single-GPU emission-order sums).  A second run forces
pair_cap below the true splat counts: every rank must raise ShardOverflowError (strict mode:
the count check lands before step() returns) instead of returning the truncated render; with only
rank 0 overflowing and lagged checks, both ranks raise for the same step at the same call.  A third
moves the camera (`set_camera`) with `rebalance_every`: the re-plan before the next step cuts
the bands for the new view, and that step's image equals the single-GPU render of it.
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import pkg, rel_l2

pytestmark = pytest.mark.gpu

WORLD = 2
W, H, P = 640, 480, 40000


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _inputs(dev):
    gr, sc = pkg("graphics"), pkg("scene")
    cam = gr.synthetic_camera(W, H)
    s = sc.make_scene(cam, P, max_sh_degree=3, seed=51)
    t = lambda a: torch.tensor(a, device=dev)
    inputs = dict(means3D=t(s.means3D), opacities=t(s.opacities), scales=t(s.scales), rotations=t(s.rotations),
                  sh_dc=t(s.sh_dc), sh_rest=t(s.sh_rest))
    return cam, inputs, t(sc.make_dL_dpix(cam, seed=52))


def _moved_camera():
    """The synthetic camera shifted 0.8 down in view space: the scene's instances crowd into the
    image's upper rows, so the balanced cuts move."""
    import math
    gr = pkg("graphics")
    fovx = math.radians(60.0)
    fovy = 2.0 * math.atan(math.tan(fovx / 2.0) * H / W)
    return gr.make_camera(np.eye(3), np.array([0.0, 0.8, 0.0]), fovx, fovy, W, H)


def _path_cams(n=20):
    """A moving camera: yaw -6..6 degrees while the view slides 0.9 down."""
    import math
    gr = pkg("graphics")
    fovx = math.radians(60.0)
    fovy = 2.0 * math.atan(math.tan(fovx / 2.0) * H / W)
    out = []
    for i in range(n):
        a = math.radians(-6.0 + 12.0 * i / (n - 1))
        Rm = np.array([[math.cos(a), 0, math.sin(a)], [0, 1, 0], [-math.sin(a), 0, math.cos(a)]])
        out.append(gr.make_camera(Rm, np.array([0.0, 0.9 * i / (n - 1), 0.0]), fovx, fovy, W, H))
    return out


def _worker(rank, port, outdir, force_pair_cap, move=False, one_rank=False, path=False):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        bands, R = pkg("bands"), pkg("rasterizer")
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        cam, inputs, dpix = _inputs(dev)
        if path:  # live re-planning over a camera path (lagged checks, no probe re-plans)
            cams = _path_cams()
            step = bands.ShardStep(R.ShardRasterizer(dev), cams[0], inputs, 3, dist, live=True).plan()
            imgs, rows = [], []
            for c in cams:
                step.set_camera(c)
                img, g, sh, st = step.step(dpix)
                imgs.append(img.cpu().numpy())
                rows.append(list(step.rows))
            step.check()
            np.savez(os.path.join(outdir, f"p{rank}.npz"), images=np.stack(imgs), rows=np.array(rows),
                     live_replans=step.live_replans, replans=step.replans)
            return
        step = bands.ShardStep(R.ShardRasterizer(dev), cam, inputs, 3, dist, strict=True,
                               rebalance_every=1 if move else 0).plan()
        if one_rank:  # only rank 0's band overflows; checks lag two steps, not strict
            step.strict = False
            if rank == 0:
                step.capacity = 1024
            guards = []
            for i in range(5):
                try:
                    step.step(dpix)
                    guards.append(int(step.overflow_guard.item()))  # the device word, before the host check
                except bands.ShardOverflowError as e:
                    np.savez(os.path.join(outdir, f"one{rank}.npz"), call=i, step=e.step, rank=e.rank,
                             band_k=e.band_k, capacity=e.capacity, guards=np.array(guards))
                    break
            return
        if move:
            step.step(dpix)  # camera A, the initial plan (no re-plan before the first step)
            rows_a = np.array(step.rows)
            step.set_camera(_moved_camera())
            img, g, sh, st = step.step(dpix)  # re-planned for camera B first
            np.savez(os.path.join(outdir, f"m{rank}.npz"), image=img.cpu().numpy(), rows_a=rows_a,
                     rows_b=np.array(step.rows), replans=step.replans, radii=sh.radii.cpu().numpy())
            return
        if force_pair_cap:
            step.pair_cap = 64
            try:
                step.step(dpix)
            except bands.ShardOverflowError as e:
                np.savez(os.path.join(outdir, f"ovf{rank}.npz"), step=e.step, counts=np.array(e.counts),
                         pair_cap=e.pair_cap)
            return
        outs = [step.step(dpix) for _ in range(2)]  # two steps: the lagged count ring is exercised
        assert int(step.overflow_guard.item()) == 0
        img, g, sh, st = outs[-1]
        assert torch.equal(img, outs[0][0])
        np.savez(os.path.join(outdir, f"r{rank}.npz"), image=img.cpu().numpy(), radii=sh.radii.cpu().numpy(),
                 g0=step.g0, g1=step.g1, rows=np.array(step.rows), pair_cap=step.pair_cap,
                 **{"grad_" + k: v.cpu().numpy() for k, v in g.items()})
    finally:
        dist.destroy_process_group()


def _run(force_pair_cap, outdir, move=False, one_rank=False, path=False):
    mp.start_processes(_worker, args=(_free_port(), outdir, force_pair_cap, move, one_rank, path), nprocs=WORLD,
                       join=True, start_method="spawn")


def test_two_process_shard_step_matches_single_gpu():
    R = pkg("rasterizer")
    dev = torch.device("cuda", 0)
    with tempfile.TemporaryDirectory() as outdir:
        _run(False, outdir)
        got = [dict(np.load(os.path.join(outdir, f"r{r}.npz"))) for r in range(WORLD)]
    cam, inputs, dpix = _inputs(dev)
    rast = R.CAbiRasterizer(dev)
    full = rast.forward(cam, **inputs, sh_degree=3)
    gf = rast.backward(full, dpix)
    want_img = full.color.cpu().numpy()
    for r in range(WORLD):
        np.testing.assert_array_equal(got[r]["image"], want_img)
    assert got[0]["rows"][1] not in (0, cam.grid[1])  # a real two-band split
    radii = np.concatenate([got[r]["radii"] for r in range(WORLD)])
    np.testing.assert_array_equal(radii, full.radii.cpu().numpy())
    for k in ("means3D", "opacities", "scales", "rotations", "sh_dc", "sh_rest", "means2D"):
        a = np.concatenate([got[r]["grad_" + k] for r in range(WORLD)])
        assert rel_l2(a, gf[k].cpu().numpy()) <= 1e-5, k


def test_two_process_overflow_raises():
    with tempfile.TemporaryDirectory() as outdir:
        _run(True, outdir)
        for r in range(WORLD):
            f = os.path.join(outdir, f"ovf{r}.npz")
            assert os.path.exists(f), f"rank {r} returned a truncated step without raising"
            e = np.load(f)
            assert int(e["step"]) == 0 and int(e["counts"].max()) > int(e["pair_cap"]) == 64


def test_two_process_camera_move_rebalances():
    R = pkg("rasterizer")
    dev = torch.device("cuda", 0)
    with tempfile.TemporaryDirectory() as outdir:
        _run(False, outdir, move=True)
        got = [dict(np.load(os.path.join(outdir, f"m{r}.npz"))) for r in range(WORLD)]
    _, inputs, _ = _inputs(dev)
    cam_b = _moved_camera()
    full = R.CAbiRasterizer(dev).forward(cam_b, **inputs, sh_degree=3)
    for r in range(WORLD):
        assert int(got[r]["replans"]) == 1
        np.testing.assert_array_equal(got[r]["rows_b"], got[0]["rows_b"])  # every rank cut alike
        np.testing.assert_array_equal(got[r]["image"], full.color.cpu().numpy())
    assert not np.array_equal(got[0]["rows_a"], got[0]["rows_b"])  # the cuts followed the view
    radii = np.concatenate([got[r]["radii"] for r in range(WORLD)])
    np.testing.assert_array_equal(radii, full.radii.cpu().numpy())


def test_two_process_overflow_agreed():
    """Only rank 0's band overflows (its capacity forced small), checks lagging two steps: both
    ranks raise ShardOverflowError at the same call, for the same step, naming rank 0 -- the
    overflow words ride in the image all-gather, so the rank whose own counts are fine is not
    left blocked in a collective."""
    with tempfile.TemporaryDirectory() as outdir:
        _run(False, outdir, one_rank=True)
        got = []
        for r in range(WORLD):
            f = os.path.join(outdir, f"one{r}.npz")
            assert os.path.exists(f), f"rank {r} never raised"
            got.append(dict(np.load(f)))
    for g in got:
        assert int(g["call"]) == 2 and int(g["step"]) == 0 and int(g["rank"]) == 0
        assert int(g["band_k"]) > int(g["capacity"]) == 1024
        # the device-side agreement word flagged both steps on BOTH ranks before the
        # lagged host check raised (a guarded optimizer step would have skipped them)
        assert g["guards"].tolist() == [1, 1]


def test_two_process_live_replan_camera_path():
    """VERDICT r04 item 6, Python step: ShardStep(live=True) over a 20-pose camera path re-cuts its
    bands from the statistics riding in the image all-gather (no probe, no extra collective): no
    overflow (check() at the end), both ranks take the same cuts, the cuts move with the view, and
    every step's image equals the single-GPU render of that camera bit for bit."""
    R = pkg("rasterizer")
    dev = torch.device("cuda", 0)
    with tempfile.TemporaryDirectory() as outdir:
        _run(False, outdir, path=True)
        got = [dict(np.load(os.path.join(outdir, f"p{r}.npz"))) for r in range(WORLD)]
    _, inputs, _ = _inputs(dev)
    rast = R.CAbiRasterizer(dev)
    np.testing.assert_array_equal(got[0]["rows"], got[1]["rows"])
    assert int(got[0]["live_replans"]) >= 2 and int(got[0]["replans"]) == 0
    assert len({tuple(r) for r in got[0]["rows"].tolist()}) >= 2
    for i, c in enumerate(_path_cams()):
        want = rast.forward(c, **inputs, sh_degree=3).color.cpu().numpy()
        for r in range(WORLD):
            np.testing.assert_array_equal(got[r]["images"][i], want, err_msg=f"rank {r} step {i}")
