"""GPU: the training loop (BASELINE configs[4], shortened), the reference's train_utils.cpp:128-145
order with the params.h:50-91 schedule, on a small synthetic multi-view scene, twice:

* the Python mirror (train_loop.train over trainer.GaussianTrainer), and
* the C++ loop (tests/cpp/train_main.cpp -> lib/gsr_train_loop over gsr::Trainer,
  csrc/torch/gsr_trainer.h): no Python in the loop, the drop-in for src/train.cpp.

3200 iterations: densification from 500 every 100, SH degree +1 at 1000 / 2000 / 3000, the first
opacity reset at 3000 and the size-threshold prune after it.  Both runs take the same cameras in
the same order and draw the split samples from the same seeded CUDA generator, and gsr::Trainer
repeats trainer.py op for op, so the bar is EXACT: the Gaussian count after every densification,
the logged losses and the final parameters are bit-identical.  The loop itself must converge
(loss down, count up, everything finite) and run every render under the lagged binning bound
(no overflow, K read back only after point-set changes)."""
import json
import math
import os
import subprocess
import tempfile

import numpy as np
import pytest
import torch

from conftest import ROOT, pkg

pytestmark = pytest.mark.gpu
EXE = os.path.join(ROOT, "3d_gaussian_splatting_amd", "lib", "gsr_train_loop")
ITERS = 3200


@pytest.fixture(scope="module")
def scene():
    return pkg("train_loop").synthetic_scene(n_gt=20000, n_init=2000, n_views=24, width=256, height=192, seed=3)


@pytest.fixture(scope="module")
def py_run(scene):
    L, T = pkg("train_loop"), pkg("trainer")
    return L.train(scene, opt=T.OptimizationParams(iterations=ITERS), max_sh_degree=3, log_every=50)


def test_python_loop_densifies_and_converges(py_run):
    res = py_run
    assert res.final_points > 2000 and res.peak_points > 2000, (res.final_points, res.num_points)
    assert len(res.num_points) >= 20 and res.num_points[-1][1] > res.num_points[0][1] >= 2000
    losses = [l for _, l, _, _ in res.loss]
    assert all(math.isfinite(v) for v in losses)
    first, last = sum(losses[:3]) / 3, sum(losses[-3:]) / 3
    assert last < 0.7 * first, (first, last)
    tr = res.trainer
    for k, v in tr.params.items():
        assert bool(torch.isfinite(v).all()), k
    assert tr.active_sh_degree == 3  # +1 at 1000, 2000, 3000
    assert res.binning_overflows == 0
    assert 1 <= res.exact_k_reads <= 2 + len(res.num_points)


def test_cpp_loop_equals_python_loop(scene, py_run):
    assert os.path.exists(EXE), "run __graft_entry__.build()"
    L, T = pkg("train_loop"), pkg("trainer")
    with tempfile.TemporaryDirectory() as d:
        fin, fres, fpar = (os.path.join(d, n) for n in ("scene.bin", "res.json", "params.bin"))
        L.write_scene(fin, scene, ITERS, T.OptimizationParams(iterations=ITERS), max_sh_degree=3, log_every=50,
                      progress_every=500)
        try:
            r = subprocess.run([EXE, fin, fres, fpar], capture_output=True, text=True, timeout=240)
        except subprocess.TimeoutExpired as e:
            pytest.fail(f"gsr_train_loop timed out; its progress:\n{e.stderr}")
        print(r.stdout, r.stderr)
        assert r.returncode == 0, r.stdout + r.stderr
        res = json.load(open(fres))
        raw = np.fromfile(fpar, np.float32)
    py = py_run
    assert res["num_points"] == [list(x) for x in py.num_points]
    assert res["final_points"] == py.final_points and res["peak_points"] == py.peak_points
    assert res["active_sh_degree"] == 3
    assert res["binning_overflows"] == 0
    cpp_loss = np.array(res["loss"], np.float64)
    py_loss = np.array(py.loss, np.float64)
    np.testing.assert_array_equal(cpp_loss[:, 0], py_loss[:, 0])
    np.testing.assert_array_equal(cpp_loss[:, 1:].astype(np.float32), py_loss[:, 1:].astype(np.float32))
    tr = py.trainer
    off = 0
    for k in ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation"):
        want = tr.params[k].cpu().numpy().ravel()
        got = raw[off:off + want.size]
        off += want.size
        np.testing.assert_array_equal(got, want, err_msg=k)
    assert off == raw.size
    print(f"C++ loop {res['iters_per_s']:.0f} it/s, Python loop {py.iters_per_s:.0f} it/s")


# ---- BASELINE configs[4] at its stated scale ------------------------------------------------
# "Full train.cpp loop, 30k iters, synthetic Mip-NeRF360-scale scene (~6M final Gaussians)": the
# C++ loop (lib/gsr_train_loop over gsr::Trainer) for the full 30 000 iterations of the params.h
# schedule at a Mip-NeRF360-like resolution, on a synthetic multi-view scene whose point count
# stays >= 5.5M to the end.  Synthetic scenes add only ~0.6M Gaussians by densification over a
# run whatever the start (profiles/r03_loop_densify_probes.jsonl), so the run
# starts near the target scale instead of growing into it; the counts are asserted and printed.
C4 = dict(n_gt=8_000_000, n_init=6_000_000, n_views=48, width=1280, height=832, iters=30_000)


def _progress_file():
    """Progress of the long run, somewhere a watchdog sees it (gpurun_out/ on the GPU box)."""
    d = os.path.join(ROOT, "gpurun_out")
    os.makedirs(d, exist_ok=True)
    return os.path.join(d, "configs4_progress.log")


@pytest.mark.timeout(900)
def test_configs4_at_scale(oracle):
    import time
    L, T = pkg("train_loop"), pkg("trainer")
    t0 = time.time()
    scene = L.synthetic_scene(C4["n_gt"], C4["n_init"], C4["n_views"], C4["width"], C4["height"], seed=7,
                              texture=1.0, gt_scale=0.012)
    cam0, gt0 = scene.cams[0], scene.gts[0].cpu().numpy()
    with tempfile.TemporaryDirectory() as d:
        fin, fres, fpar = (os.path.join(d, n) for n in ("scene.bin", "res.json", "params.bin"))
        L.write_scene(fin, scene, C4["iters"], T.OptimizationParams(iterations=C4["iters"]), max_sh_degree=3,
                      log_every=500, progress_every=1000)
        del scene
        torch.cuda.empty_cache()
        t_setup = time.time() - t0
        with open(_progress_file(), "w") as log:
            try:
                r = subprocess.run([EXE, fin, fres, fpar], stdout=log, stderr=log, timeout=600)
            except subprocess.TimeoutExpired:
                pytest.fail("configs[4] loop timed out; see " + _progress_file())
        assert r.returncode == 0, open(_progress_file()).read()
        res = json.load(open(fres))
        raw = np.fromfile(fpar, np.float32)
    n = res["final_points"]
    widths = {"xyz": 3, "f_dc": 3, "f_rest": 45, "opacity": 1, "scaling": 3, "rotation": 4}
    assert raw.size == n * sum(widths.values())
    leaves, off = {}, 0
    for k, w in widths.items():
        leaves[k] = raw[off:off + n * w].reshape(n, w)
        off += n * w
    losses = [l for _, l, _, _ in res["loss"]]
    print(f"configs[4]: {res['iterations']} iterations in {res['seconds']:.1f} s ({res['iters_per_s']:.1f} it/s) "
          f"after {t_setup:.1f} s of setup; Gaussians {C4['n_init']} -> peak {res['peak_points']} -> final {n}; "
          f"loss {losses[0]:.4f} -> {losses[-1]:.4f}; overflows {res['binning_overflows']}, "
          f"exact K reads {res['exact_k_reads']}")
    assert res["iterations"] == C4["iters"]
    assert res["binning_overflows"] == 0
    assert res["active_sh_degree"] == 3
    assert n >= 5_500_000, n
    assert all(math.isfinite(v) for v in losses)
    assert losses[-1] < 0.5 * losses[0], (losses[0], losses[-1])
    for k, v in leaves.items():
        assert np.isfinite(v).all(), k

    # the final state, one view, against the oracle (SURVEY §8d bars; test_gpu_parity.py's)
    from test_gpu_parity import _compare
    rast = pkg("rasterizer").CAbiRasterizer("cuda")
    dev = torch.device("cuda")
    tt = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)
    scales = torch.exp(tt(leaves["scaling"]))
    rots = torch.nn.functional.normalize(tt(leaves["rotation"]), dim=1)
    opac = torch.sigmoid(tt(leaves["opacity"])).reshape(-1)
    args = (cam0, tt(leaves["xyz"]), opac, scales, rots, tt(leaves["f_dc"]).reshape(n, 1, 3),
            tt(leaves["f_rest"]).reshape(n, 15, 3))
    st = rast.forward(*args, sh_degree=3)
    f = oracle.forward(*[a.cpu().numpy() if torch.is_tensor(a) else a for a in args], sh_degree=3)
    dpix = pkg("scene").make_dL_dpix(cam0, seed=8)
    worst = _compare(st, f, dpix, rast)
    psnr_gt = 10 * np.log10(1.0 / np.mean((np.clip(st.color.cpu().numpy(), 0, 1) - gt0) ** 2))
    print(f"final state vs oracle: K = {st.num_rendered}, worst gradient misses {worst}; "
          f"render vs ground truth {psnr_gt:.1f} dB")
    # the trained model reproduces its training view (33.7 dB in round 4)
    assert psnr_gt >= 30.0, psnr_gt
    # the synthetic scene's densification is net-negative: the count is met by the
    # 6.0M start, so the peak must show growth happened and the final count stay near the start
    assert res["peak_points"] > C4["n_init"], res["peak_points"]
