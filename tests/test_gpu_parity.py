"""GPU parity: the HIP kernels (through the C ABI) vs the CPU oracle on identical inputs.

Bar (north_star / SURVEY §8d):
  * discrete outputs bit-exact: radii, num_rendered, per-Gaussian depth keys and tiles, the
    sorted (tile, gid) instance list, tile ranges;
  * rendered RGB: PSNR >= 50 dB and relative L2 <= 1e-4 (tolerance written here);
  * every gradient tensor: relative L2 <= 1e-4.
Also checked against the golden fixtures (independent float64 autograd).
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, load_fixture, pkg, psnr, rel_l2

pytestmark = pytest.mark.gpu

RGB_REL, GRAD_REL, PSNR_MIN = 1e-4, 1e-4, 50.0
GRAD_KEYS = ["means2D", "opacities", "means3D", "sh_dc", "sh_rest", "scales", "rotations", "colors", "cov3D"]


@pytest.fixture(scope="module")
def rast():
    return pkg("rasterizer").CAbiRasterizer("cuda")


def _np(t):
    return t.detach().cpu().numpy()


def _compare(st, f, dpix, rast, check_grads=True):
    np.testing.assert_array_equal(_np(st.radii), f.radii)
    assert st.num_rendered == f.num_rendered
    K = st.num_rendered
    t_ref, d_ref, g_ref = f.state.sorted()
    if K:
        gid = _np(st.view(pkg("native").VIEW_SORTED_GID, torch.int32, K)).view(np.uint32)
        tile = _np(st.view(pkg("native").VIEW_SORTED_TILE, torch.int32, K)).view(np.uint32)
        np.testing.assert_array_equal(tile, t_ref)
        np.testing.assert_array_equal(gid, g_ref)
    tiles = f.state.cam.grid[0] * f.state.cam.grid[1]
    rng = _np(st.view(pkg("native").VIEW_RANGES, torch.int32, 2 * tiles)).view(np.uint32).reshape(-1, 2)
    np.testing.assert_array_equal(rng, f.state.ranges())
    color = _np(st.color)
    assert psnr(color, f.color) >= PSNR_MIN
    assert rel_l2(color, f.color) <= RGB_REL
    if not check_grads:
        return
    g_gpu = rast.backward(st, dpix)
    g_cpu = f.state.backward(dpix)
    for k in GRAD_KEYS:
        if k in g_gpu:
            a = _np(g_gpu[k]).reshape(g_cpu[k].shape)
            assert rel_l2(a, g_cpu[k]) <= GRAD_REL, (k, rel_l2(a, g_cpu[k]))


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p) for p in GOLDEN])
def test_golden_fixtures(path, rast, oracle):
    meta, cam, inp, out = load_fixture(path)
    g = inp.get
    st = rast.forward(cam, g("means3D"), g("opacities"), g("scales"), g("rotations"), g("sh_dc"), g("sh_rest"),
                      sh_degree=meta["sh_degree"], colors_precomp=g("colors_precomp"),
                      cov3D_precomp=g("cov3D_precomp"), scale_modifier=meta["scale_modifier"], bg=g("bg"),
                      debug=True)
    np.testing.assert_array_equal(_np(st.radii), out["radii"])
    assert rel_l2(_np(st.color), out["color"]) <= RGB_REL
    f = oracle.forward(cam, g("means3D"), g("opacities"), g("scales"), g("rotations"), g("sh_dc"), g("sh_rest"),
                       sh_degree=meta["sh_degree"], colors_precomp=g("colors_precomp"),
                       cov3D_precomp=g("cov3D_precomp"), scale_modifier=meta["scale_modifier"], bg=g("bg"))
    _compare(st, f, inp["dL_dpix"], rast)
    gg = rast.backward(st, inp["dL_dpix"])
    assert rel_l2(_np(gg["means2D"])[:, :2], out["grad_means2D"]) <= 2e-5
    for k in ["means3D", "opacities", "scales", "rotations", "sh_dc", "sh_rest", "colors", "cov3D"]:
        if "grad_" + k in out and out["grad_" + k].size:
            ref = out["grad_" + k]
            assert rel_l2(_np(gg[k]).reshape(ref.shape), ref) <= 2e-5, k


CONFIGS = [  # (P, W, H, active D, seed)
    (1000, 256, 256, 0, 0),      # BASELINE configs[0]: plumbing size
    (5000, 300, 200, 3, 1),      # partial tiles, SH3
    (20000, 640, 360, 2, 2),
    (100000, 800, 800, 3, 0),    # BASELINE configs[1]
]


@pytest.mark.parametrize("P,W,H,D,seed", CONFIGS)
def test_synthetic_parity(P, W, H, D, seed, rast, oracle):
    gr, sc = pkg("graphics"), pkg("scene")
    cam = gr.synthetic_camera(W, H)
    s = sc.make_scene(cam, P, max_sh_degree=3, seed=seed)
    dpix = sc.make_dL_dpix(cam, seed=seed + 1)
    args = (cam, s.means3D, s.opacities, s.scales, s.rotations, s.sh_dc, s.sh_rest)
    st = rast.forward(*args, sh_degree=D)
    f = oracle.forward(*args, sh_degree=D)
    # per-Gaussian keys bit-exact
    dk = _np(st.view(pkg("native").VIEW_DEPTH_KEY, torch.int32, P)).view(np.uint32)
    pre = f.state.preprocess()
    vis = f.radii > 0
    np.testing.assert_array_equal(dk[vis], pre["depth"][vis].view(np.uint32))
    assert np.all(dk[~vis] == 0xFFFFFFFF)
    tt = _np(st.view(pkg("native").VIEW_TILES_TOUCHED, torch.int32, P)).view(np.uint32)
    np.testing.assert_array_equal(tt, pre["tiles_touched"])
    _compare(st, f, dpix, rast)


def test_band_sharded_equals_full(rast):
    """Tile-row bands (multi-GPU shard unit): image bands and summed grad2d equal the full run."""
    gr, sc = pkg("graphics"), pkg("scene")
    cam = gr.synthetic_camera(320, 240)
    s = sc.make_scene(cam, 8000, max_sh_degree=3, seed=4)
    dpix = sc.make_dL_dpix(cam, seed=5)
    args = (cam, s.means3D, s.opacities, s.scales, s.rotations, s.sh_dc, s.sh_rest)
    full = rast.forward(*args, sh_degree=3)
    g_full = rast.backward(full, dpix)
    gy = cam.grid[1]
    bands = [(0, 4), (4, 9), (9, gy)]
    img = torch.zeros_like(full.color)
    grad2d = None
    for y0, y1 in bands:
        st = rast.forward(*args, sh_degree=3, tile_rows=(y0, y1))
        img[:, y0 * 16:y1 * 16] = st.color[:, y0 * 16:y1 * 16]
        # the band ranks exactly its candidates (Gaussians with tiles in the band): in gid
        # order (shipped binning, per-tile depth order) or depth-sorted (GSR_BIN_VARIANT=0)
        native = pkg("native")
        nr = st.buffers.num_ranked
        cand = _np(st.view(native.VIEW_GID_BY_RANK, torch.int32, nr)).astype(np.int64)
        tt = _np(st.view(native.VIEW_TILES_TOUCHED, torch.int32, s.P))
        key = _np(st.view(native.VIEW_DEPTH_KEY, torch.int32, s.P)).view(np.uint32)
        np.testing.assert_array_equal(np.sort(cand), np.nonzero(tt)[0])
        if os.environ.get("GSR_BIN_VARIANT", "2") == "0":
            assert np.all(np.diff(key[cand].astype(np.int64)) >= 0)
        else:
            assert np.all(np.diff(cand) > 0)
        g2 = rast.backward_blend(st, dpix)
        grad2d = g2 if grad2d is None else grad2d + g2
        last = st
    assert torch.equal(img, full.color)
    g = rast.backward_preprocess(last, grad2d)
    for k in ["means2D", "opacities", "means3D", "sh_dc", "sh_rest", "scales", "rotations"]:
        assert rel_l2(_np(g[k]), _np(g_full[k])) <= 1e-5, k


def test_band_only_flag(rast):
    """GSR_FLAG_BAND_ONLY (the multi-GPU path) leaves out-of-band pixels and non-candidate
    grad2d rows unwritten; the band rows and candidate rows equal the default run's."""
    gr, sc, native = pkg("graphics"), pkg("scene"), pkg("native")
    cam = gr.synthetic_camera(320, 240)
    s = sc.make_scene(cam, 8000, max_sh_degree=3, seed=6)
    dpix = sc.make_dL_dpix(cam, seed=7)
    args = (cam, s.means3D, s.opacities, s.scales, s.rotations, s.sh_dc, s.sh_rest)
    y0, y1 = 5, 10
    ref = rast.forward(*args, sh_degree=3, tile_rows=(y0, y1))
    g_ref = rast.backward_blend(ref, dpix)
    st = rast.forward(*args, sh_degree=3, tile_rows=(y0, y1), band_only=True)
    assert torch.equal(st.color[:, y0 * 16:y1 * 16], ref.color[:, y0 * 16:y1 * 16])
    out = torch.full_like(g_ref, float("nan"))
    g2 = rast.backward_blend(st, dpix, out=out)
    cand = st.view(native.VIEW_GID_BY_RANK, torch.int32, st.buffers.num_ranked).long()
    assert torch.equal(g2[cand], g_ref[cand])
    rest = torch.ones(s.P, dtype=torch.bool, device=g2.device)
    rest[cand] = False
    assert bool(torch.isnan(g2[rest]).all())  # untouched
    assert float(g_ref[rest].abs().max()) == 0.0


def test_dense_tiles_sort_paths(rast, oracle):
    """Tiles holding more instances than the per-tile depth sort's shared-memory form takes:
    (a) 60k Gaussians on a 64x48 image (12 tiles, ~10^4 instances each) exercise the
    global-memory form beyond 8192; (b) a cluster of 6000 Gaussians in the middle of a
    sparse 256x256 scene overflows a 1024-slot tile into the 8192-slot LDS form.  Canonical
    order, ranges and outputs must still match the oracle."""
    gr, sc = pkg("graphics"), pkg("scene")
    cam = gr.synthetic_camera(64, 48)
    s = sc.make_scene(cam, 60000, max_sh_degree=1, seed=11)
    args = (cam, s.means3D, s.opacities, s.scales, s.rotations, s.sh_dc, s.sh_rest)
    st = rast.forward(*args, sh_degree=1)
    f = oracle.forward(*args, sh_degree=1)
    tiles = cam.grid[0] * cam.grid[1]
    rng = _np(st.view(pkg("native").VIEW_RANGES, torch.int32, 2 * tiles)).view(np.uint32).reshape(-1, 2)
    assert int((rng[:, 1] - rng[:, 0]).max()) > 8192
    _compare(st, f, sc.make_dL_dpix(cam, seed=12), rast)

    cam = gr.synthetic_camera(256, 256)
    s = sc.make_scene(cam, 20000, max_sh_degree=1, seed=13)
    s.means3D[:6000, :2] *= 0.02  # pile 6000 Gaussians onto the centre tiles
    args = (cam, s.means3D, s.opacities, s.scales, s.rotations, s.sh_dc, s.sh_rest)
    st = rast.forward(*args, sh_degree=1)
    f = oracle.forward(*args, sh_degree=1)
    tiles = cam.grid[0] * cam.grid[1]
    rng = _np(st.view(pkg("native").VIEW_RANGES, torch.int32, 2 * tiles)).view(np.uint32).reshape(-1, 2)
    n = rng[:, 1] - rng[:, 0]
    assert 1024 < int(n.max()) <= 8192 and float(n.mean()) < 1024
    _compare(st, f, sc.make_dL_dpix(cam, seed=14), rast)


def test_empty_and_culled(rast):
    gr, sc = pkg("graphics"), pkg("scene")
    cam = gr.synthetic_camera(64, 48)
    s = sc.make_scene(cam, 50, max_sh_degree=1)
    means = s.means3D.copy()
    means[:, 2] = -2.0
    st = rast.forward(cam, means, s.opacities, s.scales, s.rotations, s.sh_dc, s.sh_rest, sh_degree=1,
                      bg=(0.1, 0.2, 0.3), debug=True)
    assert st.num_rendered == 0
    c = _np(st.color)
    np.testing.assert_allclose(c.reshape(3, -1), np.repeat([[0.1], [0.2], [0.3]], 64 * 48, 1), atol=1e-7)
    g = rast.backward(st, np.ones((3, 48, 64), np.float32))
    assert all(float(v.abs().max()) == 0.0 for v in g.values())
    # P = 0
    st0 = rast.forward(cam, np.zeros((0, 3)), np.zeros(0), np.zeros((0, 3)), np.zeros((0, 4)),
                       np.zeros((0, 1, 3)), None, sh_degree=0, bg=(1, 1, 1))
    assert float(st0.color.min()) == 1.0


def test_deterministic(rast):
    gr, sc = pkg("graphics"), pkg("scene")
    cam = gr.synthetic_camera(256, 192)
    s = sc.make_scene(cam, 10000, max_sh_degree=3, seed=9)
    dpix = sc.make_dL_dpix(cam)
    args = (cam, s.means3D, s.opacities, s.scales, s.rotations, s.sh_dc, s.sh_rest)
    a = rast.forward(*args, sh_degree=3)
    b = rast.forward(*args, sh_degree=3)
    assert torch.equal(a.color, b.color)
    ga, gb = rast.backward(a, dpix), rast.backward(b, dpix)
    for k in ga:
        assert torch.equal(ga[k], gb[k]), k


def test_full_size_properties(rast):
    """1M Gaussians at 1080p (BASELINE configs[2]): size-independent properties -- canonical
    sortedness of (tile, depth bits, gid), ranges consistent, transmittance in [0,1]."""
    gr, sc = pkg("graphics"), pkg("scene")
    native = pkg("native")
    cam = gr.synthetic_camera(1920, 1080)
    s = sc.make_scene(cam, 1_000_000, max_sh_degree=3, seed=0)
    st = rast.forward(cam, s.means3D, s.opacities, s.scales, s.rotations, s.sh_dc, s.sh_rest, sh_degree=3)
    K = st.num_rendered
    assert K > 1_000_000
    tile = st.view(native.VIEW_SORTED_TILE, torch.int32, K).to(torch.int64)
    gid = st.view(native.VIEW_SORTED_GID, torch.int32, K).to(torch.int64)
    dk = st.view(native.VIEW_DEPTH_KEY, torch.int32, s.P).to(torch.int64) & 0xFFFFFFFF
    key = tile * (1 << 32) + dk[gid]
    assert bool((key[1:] >= key[:-1]).all())
    tie = key[1:] == key[:-1]
    assert bool((gid[1:][tie] > gid[:-1][tie]).all())
    assert int((st.radii > 0).sum()) == int(torch.bincount(gid, minlength=s.P).gt(0).sum())
    T = st.view(native.VIEW_FINAL_T, torch.float32, cam.width * cam.height)
    assert float(T.min()) >= 0.0 and float(T.max()) <= 1.0
    assert bool(torch.isfinite(st.color).all())


@pytest.mark.gpu
def test_backward_preprocess_range_matches_full():
    """B2 on Gaussian slices (multi-GPU sharded leaf gradients) equals the slices of the
    full B2, bit for bit (same per-Gaussian arithmetic)."""
    R, gr, sc = pkg("rasterizer"), pkg("graphics"), pkg("scene")
    import torch
    dev = torch.device("cuda", 0)
    cam = gr.synthetic_camera(320, 240)
    scene = sc.make_scene(cam, 5000, max_sh_degree=3, seed=7)
    dpix = torch.tensor(sc.make_dL_dpix(cam, seed=8), device=dev)
    t = lambda a: torch.tensor(a, device=dev)
    rast = R.CAbiRasterizer(dev)
    st = rast.forward(cam, means3D=t(scene.means3D), opacities=t(scene.opacities), scales=t(scene.scales),
                      rotations=t(scene.rotations), sh_dc=t(scene.sh_dc), sh_rest=t(scene.sh_rest), sh_degree=3)
    g2 = rast.backward_blend(st, dpix)
    full = rast.backward_preprocess(st, g2)
    P = scene.P
    for g0, g1 in ((0, 1234), (1234, 4999), (4999, 5000), (0, P)):
        part = rast.backward_preprocess_range(st, g0, g1, g2[g0:g1])
        for k, v in part.items():
            assert torch.equal(v, full[k][g0:g1]), (k, g0, g1)


@pytest.mark.gpu
def test_fused_gather_backward_matches_two_kernels(monkeypatch):
    """gsr_backward's fused gather + B2 (GSR_FUSE_GATHER=1; full image, gid-order ranking)
    equals B1 -> grad2d -> B2 through gsr_backward_blend / gsr_backward_preprocess, bit for bit."""
    monkeypatch.setenv("GSR_FUSE_GATHER", "1")
    R, gr, sc = pkg("rasterizer"), pkg("graphics"), pkg("scene")
    dev = torch.device("cuda", 0)
    for D, P, (W, H) in ((3, 20000, (320, 240)), (0, 3000, (200, 120))):
        cam = gr.synthetic_camera(W, H)
        s = sc.make_scene(cam, P, max_sh_degree=3, seed=17)
        dpix = torch.tensor(sc.make_dL_dpix(cam, seed=18), device=dev)
        rast = R.CAbiRasterizer(dev)
        st = rast.forward(cam, s.means3D, s.opacities, s.scales, s.rotations, s.sh_dc, s.sh_rest, sh_degree=D)
        fused = rast.backward(st, dpix)
        two = rast.backward_preprocess(st, rast.backward_blend(st, dpix))
        for k, v in fused.items():
            assert torch.equal(v, two[k]), (D, k)


@pytest.mark.gpu
def test_f6_stripe_variants_bit_identical(monkeypatch):
    """F6's shipped branchless stripe pair (GSR_F6_BRANCHLESS=1) and the per-stripe branch
    (=0) give the same image and, through F6's chunk checkpoints, the same gradients, bit for
    bit: a culled stripe's pixels get alpha 0, which leaves C and T unchanged."""
    R, gr, sc = pkg("rasterizer"), pkg("graphics"), pkg("scene")
    dev = torch.device("cuda", 0)
    cam = gr.synthetic_camera(640, 480)
    s = sc.make_scene(cam, 60000, max_sh_degree=3, seed=23)
    dpix = torch.tensor(sc.make_dL_dpix(cam, seed=24), device=dev)
    out = {}
    for v in ("0", "1"):
        monkeypatch.setenv("GSR_F6_BRANCHLESS", v)
        rast = R.CAbiRasterizer(dev)
        st = rast.forward(cam, s.means3D, s.opacities, s.scales, s.rotations, s.sh_dc, s.sh_rest, sh_degree=3)
        out[v] = (st.color.clone(), rast.backward(st, dpix))
    assert torch.equal(out["0"][0], out["1"][0])
    for k, g in out["0"][1].items():
        assert torch.equal(g, out["1"][1][k]), k
