"""GPU: point-cloud initialisation and checkpoints.

  * gsr_knn_mean_dist2 (exact 3-NN mean squared distance, the upstream distCUDA2 quantity)
    against scipy's cKDTree in float64 -- relative tolerance 1e-5 (f32 distances);
  * GaussianTrainer.from_point_cloud against the upstream create_from_pcd formulas;
  * capture -> restore -> identical continued training (bitwise: every kernel is
    deterministic), and save_ply -> from_ply round trip.
"""
import numpy as np
import pytest
import torch

from conftest import pkg

pytestmark = pytest.mark.gpu
KNN_RTOL = 1e-5


def _ref_knn(pts):
    from scipy.spatial import cKDTree
    p = pts.astype(np.float64)
    d, _ = cKDTree(p).query(p, k=4)
    return (d[:, 1:] ** 2).mean(1)


def _knn(pts):
    k = pkg("trainer").TrainKernels("cuda")
    return k.knn_mean_dist2(torch.tensor(pts, dtype=torch.float32, device="cuda")).cpu().numpy()


@pytest.mark.parametrize("case", ["gauss", "clusters", "duplicates", "plane", "large"])
def test_knn_matches_kdtree(case):
    rng = np.random.default_rng(7)
    if case == "gauss":
        pts = rng.normal(size=(5000, 3))
    elif case == "clusters":  # very uneven density: most boxes skipped, some scanned a lot
        c = rng.normal(size=(20, 3)) * 10
        pts = c[rng.integers(0, 20, 8000)] + rng.normal(size=(8000, 3)) * rng.choice([0.01, 0.5], 8000)[:, None]
    elif case == "duplicates":  # exact repeats: zero distances
        base = rng.normal(size=(700, 3))
        pts = np.concatenate([base, base[:300], base[:50]])
    elif case == "plane":  # a degenerate axis (zero extent in z)
        pts = np.concatenate([rng.uniform(-1, 1, size=(3000, 2)), np.zeros((3000, 1))], 1)
    else:  # ~COLMAP scale
        pts = rng.uniform(-5, 5, size=(200_000, 3)) * np.array([1.0, 0.5, 2.0])
    pts = pts.astype(np.float32)
    np.testing.assert_allclose(_knn(pts), _ref_knn(pts), rtol=KNN_RTOL, atol=1e-12)


def test_knn_small_n():
    # fewer than 3 other points: the missing neighbours count as FLT_MAX (upstream's initial
    # best distances), so the mean is huge (clamped, then log'd, by create_from_pcd)
    fmax = np.float32(np.finfo(np.float32).max)
    np.testing.assert_allclose(_knn(np.zeros((3, 3), np.float32)), np.float32(fmax / np.float32(3)), rtol=1e-6)
    assert np.all(np.isinf(_knn(np.zeros((1, 3), np.float32))))
    pts = np.array([[0, 0, 0], [1, 0, 0], [0, 2, 0], [0, 0, 3]], np.float32)
    np.testing.assert_allclose(_knn(pts), _ref_knn(pts), rtol=KNN_RTOL)
    assert _knn(np.zeros((0, 3), np.float32)).size == 0


def test_from_point_cloud_matches_create_from_pcd():
    tr_mod, io = pkg("trainer"), pkg("scene_io")
    rng = np.random.default_rng(8)
    pts = rng.normal(size=(3000, 3)).astype(np.float32)
    col = rng.uniform(size=(3000, 3)).astype(np.float32)
    tr = tr_mod.GaussianTrainer.from_point_cloud(pts, col, max_sh_degree=3, spatial_lr_scale=2.5)
    p = {k: v.cpu().numpy() for k, v in tr.params.items()}
    d2 = np.maximum(_ref_knn(pts), 1e-7)
    np.testing.assert_allclose(p["scaling"], np.repeat(np.log(np.sqrt(d2))[:, None], 3, 1), rtol=1e-5, atol=1e-6)
    np.testing.assert_array_equal(p["xyz"], pts)
    np.testing.assert_allclose(p["f_dc"][:, 0], io.rgb2sh(col), rtol=1e-6, atol=1e-6)
    assert p["f_rest"].shape == (3000, 15, 3) and not p["f_rest"].any()
    np.testing.assert_array_equal(p["rotation"], np.tile([1, 0, 0, 0], (3000, 1)))
    np.testing.assert_allclose(p["opacity"], np.log(0.1 / 0.9), rtol=1e-6)
    assert tr.spatial_lr_scale == 2.5 and tr.lr["xyz"] == pytest.approx(tr.opt.position_lr_init * 2.5)


def _trainer(seed=0):
    gr, sc, tr_mod = pkg("graphics"), pkg("scene"), pkg("trainer")
    cam = gr.synthetic_camera(160, 120)
    s = sc.make_scene(cam, 3000, max_sh_degree=3, seed=seed)
    tr = tr_mod.GaussianTrainer(s.means3D, s.sh_dc, s.sh_rest, s.raw_opacities, s.raw_scales, s.raw_rotations,
                                max_sh_degree=3, spatial_lr_scale=1.3)
    gt = torch.tensor(sc.make_dL_dpix(cam, seed=3), device="cuda") * 0.5 + 0.5
    return tr, cam, gt


def test_capture_restore_continues_identically(tmp_path):
    a, cam, gt = _trainer()
    for it in range(1, 4):
        a.step(it, cam, gt, densify=False)
    path = str(tmp_path / "chkpnt.pth")
    a.capture(path)
    b, _, _ = _trainer(seed=5)  # a different initial state: restore must replace all of it
    b.restore(path)
    assert b.active_sh_degree == a.active_sh_degree and b.steps == a.steps
    for it in range(4, 6):
        a.step(it, cam, gt, densify=False)
        b.step(it, cam, gt, densify=False)
    for k in a.params:
        assert torch.equal(a.params[k], b.params[k]), k
        assert torch.equal(a.exp_avg_sq[k], b.exp_avg_sq[k]), k
    assert torch.equal(a.xyz_gradient_accum, b.xyz_gradient_accum)


def test_ply_round_trip(tmp_path):
    a, _, _ = _trainer()
    path = str(tmp_path / "point_cloud.ply")
    a.save_ply(path)
    b = pkg("trainer").GaussianTrainer.from_ply(path, max_sh_degree=3)
    for k in a.params:
        assert torch.equal(a.params[k], b.params[k]), k
    assert b.active_sh_degree == 3
