"""CPU oracle pinned against the committed golden fixtures (independent dense torch-autograd
restatement, tests/golden/gen_golden.py) plus size-independent properties of its output."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, ROOT, load_fixture, pkg, rel_l2

GRAD_KEYS = ["means3D", "opacities", "scales", "rotations", "sh_dc", "sh_rest", "colors", "cov3D"]


def _run(oracle, cam, inp, meta, tile_rows=None):
    g = inp.get
    return oracle.forward(cam, g("means3D"), g("opacities"), g("scales"), g("rotations"), g("sh_dc"),
                          g("sh_rest"), sh_degree=meta["sh_degree"], colors_precomp=g("colors_precomp"),
                          cov3D_precomp=g("cov3D_precomp"), scale_modifier=meta["scale_modifier"],
                          bg=g("bg"), tile_rows=tile_rows)


def test_fixture_manifest():
    with open(os.path.join(ROOT, "tests", "golden", "MANIFEST.json")) as fh:
        man = json.load(fh)
    assert set(man) == {os.path.basename(p) for p in GOLDEN}
    assert len(GOLDEN) >= 5


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p) for p in GOLDEN])
def test_oracle_matches_golden(path, oracle):
    meta, cam, inp, out = load_fixture(path)
    f = _run(oracle, cam, inp, meta)
    # discrete decisions: exact
    np.testing.assert_array_equal(f.radii, out["radii"])
    T, n = f.state.pixel_state()
    np.testing.assert_array_equal(n, out["n_contrib"])
    # values: float32 oracle vs float64 autograd
    assert rel_l2(f.color, out["color"]) < 1e-5
    assert rel_l2(T, out["final_T"]) < 1e-5
    g = f.state.backward(inp["dL_dpix"])
    assert rel_l2(g["means2D"][:, :2], out["grad_means2D"]) < 2e-5
    for k in GRAD_KEYS:
        if "grad_" + k in out:
            ref = out["grad_" + k]
            assert rel_l2(g[k].reshape(ref.shape), ref) < 2e-5, k


def _elem(a, b, rel, floor_frac):
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    f = floor_frac * float(np.abs(b).max())
    return float((np.abs(a - b) / (rel * np.maximum(np.abs(b), f))).max()) if f > 0 else 0.0


def test_oracle_elementwise_floor_vs_fp64(oracle):
    """Where f32 arithmetic ends: the oracle against the independent fp64 autograd fixtures.
    RGB meets SURVEY §8d's element-wise bound |a - b| <= 1e-4 max(|b|, 1e-3 max|b|) with room to
    spare; gradients do not (cancelling sums over many pairs: up to 5x over it), but all meet
    |a - b| <= 1e-3 max(|b|, 1e-2 max|b|) -- the element-wise bound the GPU parity tests apply to
    gradients (tests/test_gpu_parity.py ELEM_GRAD)."""
    worst_spec = 0.0
    for path in GOLDEN:
        meta, cam, inp, out = load_fixture(path)
        f = _run(oracle, cam, inp, meta)
        assert _elem(f.color, out["color"], 1e-4, 1e-3) <= 1.0
        g = f.state.backward(inp["dL_dpix"])
        for k in GRAD_KEYS:
            if "grad_" + k in out and out["grad_" + k].size:
                ref = out["grad_" + k]
                a = g[k].reshape(ref.shape)
                assert _elem(a, ref, 1e-3, 1e-2) <= 1.0, (path, k)
                worst_spec = max(worst_spec, _elem(a, ref, 1e-4, 1e-3))
    assert worst_spec > 1.0  # the spec bound is beyond f32 for gradients (documents the floor)


def _scene(P, W, H, D=3, seed=0):
    gr, sc = pkg("graphics"), pkg("scene")
    cam = gr.synthetic_camera(W, H)
    return cam, sc.make_scene(cam, P, max_sh_degree=3, seed=seed)


def test_canonical_sort_order(oracle):
    cam, s = _scene(2000, 160, 128)
    f = oracle.forward(cam, s.means3D, s.opacities, s.scales, s.rotations, s.sh_dc, s.sh_rest, sh_degree=3)
    t, d, g = f.state.sorted()
    key = t.astype(np.uint64) << np.uint64(32) | d.astype(np.uint64)
    assert np.all(np.diff(key.astype(np.float64)) >= 0)
    tie = (t[1:] == t[:-1]) & (d[1:] == d[:-1])
    assert np.all(g[1:][tie] > g[:-1][tie])
    r = f.state.ranges()
    assert r[:, 1].max() == f.num_rendered
    for tile in np.nonzero(r[:, 1] > r[:, 0])[0][:50]:
        assert np.all(t[r[tile, 0]:r[tile, 1]] == tile)


def test_band_union_equals_full(oracle):
    """Tile-row bands (the multi-GPU shard unit) reassemble the full image exactly."""
    cam, s = _scene(1500, 128, 96)
    args = (cam, s.means3D, s.opacities, s.scales, s.rotations, s.sh_dc, s.sh_rest)
    full = oracle.forward(*args, sh_degree=2)
    gy = cam.grid[1]
    img = np.zeros_like(full.color)
    for y0, y1 in [(0, 2), (2, 3), (3, gy)]:
        part = oracle.forward(*args, sh_degree=2, tile_rows=(y0, y1))
        img[:, y0 * 16:y1 * 16] = part.color[:, y0 * 16:y1 * 16]
        np.testing.assert_array_equal(part.radii, full.radii)
    np.testing.assert_array_equal(img, full.color)


def test_all_culled_gives_background(oracle):
    cam, s = _scene(100, 64, 64)
    means = s.means3D.copy()
    means[:, 2] = -1.0  # behind the camera
    f = oracle.forward(cam, means, s.opacities, s.scales, s.rotations, s.sh_dc, s.sh_rest, sh_degree=3,
                       bg=(0.2, 0.4, 0.6))
    assert f.num_rendered == 0
    assert np.all(f.radii == 0)
    np.testing.assert_allclose(f.color.reshape(3, -1).mean(1), [0.2, 0.4, 0.6], atol=1e-7)
    g = f.state.backward(np.ones((3, 64, 64), np.float32))
    assert all(np.all(v == 0) for v in g.values())


def test_single_gaussian_closed_form(oracle):
    """One isotropic Gaussian at the image centre: pixel value = o*exp(power)*rgb exactly."""
    gr = pkg("graphics")
    cam = gr.synthetic_camera(64, 64)
    z = 5.0
    f = oracle.forward(cam, np.array([[0.0, 0.0, z]]), np.array([0.8]), scales=np.array([[0.05] * 3]),
                       rotations=np.array([[1.0, 0, 0, 0]]), colors_precomp=np.array([[1.0, 0.5, 0.25]]))
    assert f.num_rendered > 0
    fx = 64 / (2 * cam.tanfovx)
    var = (fx * 0.05 / z) ** 2 + 0.3
    cx = (64 - 1) * 0.5
    for px, py in [(31, 31), (35, 30), (28, 33)]:
        d2 = (cx - px) ** 2 + (cx - py) ** 2
        alpha = 0.8 * np.exp(-0.5 * d2 / var)
        if alpha >= 1 / 255:
            assert f.color[0, py, px] == pytest.approx(alpha, rel=1e-4)
            assert f.color[1, py, px] == pytest.approx(0.5 * alpha, rel=1e-4)


def test_occlusion_order(oracle):
    """Nearer Gaussian composites first regardless of input order."""
    gr = pkg("graphics")
    cam = gr.synthetic_camera(32, 32)
    means = np.array([[0.0, 0.0, 6.0], [0.0, 0.0, 3.0]])
    cols = np.array([[1.0, 0, 0], [0, 1.0, 0]])
    f = oracle.forward(cam, means, np.array([0.9, 0.9]), scales=np.array([[0.5] * 3, [0.25] * 3]),
                       rotations=np.array([[1.0, 0, 0, 0]] * 2), colors_precomp=cols)
    c = f.color[:, 15, 15]
    assert c[1] > c[0] > 0  # green (near) dominates red (far)
