"""GPU: views mode -- V same-size cameras in ONE pass, one launch per stage (SURVEY §8f row 4,
gsr_forward_views / gsr_backward_views).

The pass must give, view by view, exactly what gsr_forward / gsr_backward give for that camera
alone: colour, radii, means2D / conic gradients bit for bit, and leaf gradients bit for bit
equal to the per-view results added in view order ((g0 + g1) + g2 ...).  A tile belongs to one
view's band of the tall binning, and the canonical (tile, depth, Gaussian) order is the same
whether the entries come from the global depth pre-sort (V * P >= 2^19 + 1) or the per-tile
depth sort, so even a pass that switches sort paths is bit-identical.
"""
import math

import numpy as np
import pytest
import torch

from conftest import pkg, psnr, rel_l2

pytestmark = pytest.mark.gpu


def _rot_y(deg):
    a = math.radians(deg)
    return np.array([[math.cos(a), 0, math.sin(a)], [0, 1, 0], [-math.sin(a), 0, math.cos(a)]])


def _cams(w, h, n):
    gr = pkg("graphics")
    poses = [(0, (0, 0, 0)), (8, (0.3, 0, 0)), (-12, (0, 0.2, 0.5)), (4, (0, 0, -0.5)), (90, (0, 0, 0)),
             (20, (-0.2, 0.1, 0)), (-5, (0.1, -0.1, 0.2)), (2, (0, 0, 0.3))]
    fx = math.radians(60.0)
    fy = 2 * math.atan(math.tan(fx / 2) * h / w)
    return [gr.make_camera(_rot_y(d), np.array(t, float), fx, fy, w, h) for d, t in poses[:n]]


def _scene(P, seed, w=320, h=240):
    gr, sc = pkg("graphics"), pkg("scene")
    s = sc.make_scene(gr.synthetic_camera(w, h), P, max_sh_degree=3, seed=seed)
    return (s.means3D, s.opacities, s.scales, s.rotations, s.sh_dc, s.sh_rest)


def _check(rast, cams, args, bg=(0.1, 0.2, 0.3)):
    V = len(cams)
    st = rast.forward_views(cams, *args, sh_degree=3, bg=bg)
    H, W = cams[0].height, cams[0].width
    assert st.color.shape == (V, 3, H, W)
    gen = torch.Generator("cuda").manual_seed(5)
    dpix = torch.rand((V, 3, H, W), device="cuda", generator=gen)
    gv = rast.backward_views(st, dpix)
    total, leaf = 0, None
    for v, cam in enumerate(cams):
        a = rast.forward(cam, *args, sh_degree=3, bg=bg)
        assert torch.equal(a.color, st.color[v]), v
        assert torch.equal(a.radii, st.radii[v]), v
        total += a.num_rendered
        ga = rast.backward(a, dpix[v])
        for k in ("means2D", "conic"):
            assert torch.equal(ga[k], gv[k][v]), (k, v)
        leaf = {k: t.clone() for k, t in ga.items() if k not in ("means2D", "conic")} if leaf is None else \
            {k: leaf[k] + ga[k] for k in leaf}
    assert st.num_rendered == total
    for k in leaf:
        assert torch.equal(leaf[k], gv[k]), k
    return st


def test_views_equal_single_views():
    rast = pkg("rasterizer").CAbiRasterizer("cuda")
    cams = _cams(320, 250, 5)  # 250 rows: the last tile row of every view is part padding
    _check(rast, cams, _scene(20000, 21))


def test_views_presort_switch():
    """V * P crosses the pre-sort threshold, each view alone does not."""
    native = pkg("native")
    rast = pkg("rasterizer").CAbiRasterizer("cuda")
    cams = _cams(400, 304, 4)
    P = 600000
    assert P < (1 << 21) + 1 <= 4 * P  # gsr_internal.h GSR_PRESORT_MIN
    _check(rast, cams, _scene(P, 22, 400, 304))
    assert native.GSR_MAX_VIEWS == 8


def test_views_full_and_one():
    rast = pkg("rasterizer").CAbiRasterizer("cuda")
    args = _scene(12000, 23, 192, 128)
    _check(rast, _cams(192, 128, 8), args)
    _check(rast, _cams(192, 128, 1), args)


def test_views_bounded_count():
    """Under a binning bound K stays on the device; ViewsState.num_rendered reads it back through
    the pass's tall camera, and a bound below K is reported as an overflow."""
    rast = pkg("rasterizer").CAbiRasterizer("cuda")
    args = _scene(20000, 25, 320, 240)
    cams = _cams(320, 240, 3)
    exact = rast.forward_views(cams, *args, sh_degree=3)
    K = exact.num_rendered
    bounded = rast.forward_views(cams, *args, sh_degree=3, max_rendered=K + 100)
    assert bounded.num_rendered == K
    assert torch.equal(bounded.color, exact.color)
    short = rast.forward_views(cams, *args, sh_degree=3, max_rendered=max(K // 2, 1))
    with pytest.raises(OverflowError):
        short.num_rendered


def test_views_limits():
    rast = pkg("rasterizer").CAbiRasterizer("cuda")
    args = _scene(2000, 24, 128, 96)
    cams = _cams(128, 96, 2)
    with pytest.raises(RuntimeError, match="views"):
        rast.forward_views(cams * 5, *args, sh_degree=3)  # 10 > GSR_MAX_VIEWS
    other = _cams(96, 96, 1)
    with pytest.raises(RuntimeError, match="every view"):
        rast.forward_views(cams + other, *args, sh_degree=3)
    empty = rast.forward_views(cams, np.zeros((0, 3)), np.zeros(0), np.zeros((0, 3)), np.zeros((0, 4)),
                               np.zeros((0, 1, 3)), None, sh_degree=0, bg=(1, 1, 1))
    assert float(empty.color.min()) == 1.0 and float(empty.color.max()) == 1.0


def test_views_vs_oracle(oracle):
    """Views mode against the CPU oracle, view by view (§8f row 4; the camera
    matrices of camera.cpp:66-71 / graphics_utils.cpp:32-72 through graphics.make_camera): the
    eight poses of _cams -- yaw up to 90 degrees, translations -- at 320 x 250 (the last tile row
    of every view is part padding), coloured background.

    Bars: radii, the sorted (tile, Gaussian) list and the tile ranges bit-exact per
    view (the pass's tall grid: view v's tiles are v * T + t and its entries v * P + g, so view
    v's segment of the pass's list is the oracle's list shifted); per view RGB PSNR >= 50 dB and
    rel-L2 <= 1e-4, means2D / conic gradients rel-L2 <= 1e-4; the summed leaf gradients within
    1e-4 rel-L2 of the sum of the oracle's per-view gradients."""
    native = pkg("native")
    rast = pkg("rasterizer").CAbiRasterizer("cuda")
    W, H, P = 320, 250, 20000
    cams = _cams(W, H, 8)
    args = _scene(P, 31, W, H)
    bg = (0.1, 0.2, 0.3)
    st = rast.forward_views(cams, *args, sh_degree=3, bg=bg)
    V = len(cams)
    gx, gy = (W + 15) // 16, (H + 15) // 16
    T = gx * gy
    K = st.num_rendered
    tiles = st.view(native.VIEW_SORTED_TILE, torch.int32, K).cpu().numpy().view(np.uint32)
    gids = st.view(native.VIEW_SORTED_GID, torch.int32, K).cpu().numpy().view(np.uint32)
    ranges = st.view(native.VIEW_RANGES, torch.int32, 2 * V * T).cpu().numpy().view(np.uint32).reshape(V * T, 2)
    gen = np.random.default_rng(32)
    dpix = gen.random((V, 3, H, W), dtype=np.float32)
    gv = rast.backward_views(st, torch.tensor(dpix, device="cuda"))
    col = st.color.cpu().numpy()
    radii = st.radii.cpu().numpy()
    leaf_sum, k0, seen = None, 0, 0
    for v, cam in enumerate(cams):
        f = oracle.forward(cam, *args, sh_degree=3, bg=bg)
        np.testing.assert_array_equal(radii[v], f.radii, err_msg=f"radii, view {v}")
        kv = int(f.num_rendered)
        t_ref, _, g_ref = f.state.sorted()
        np.testing.assert_array_equal(tiles[k0:k0 + kv], t_ref + v * T, err_msg=f"sorted tiles, view {v}")
        np.testing.assert_array_equal(gids[k0:k0 + kv], g_ref + v * P, err_msg=f"sorted gids, view {v}")
        r_ref = f.state.ranges()
        r_got = ranges[v * T:(v + 1) * T]
        live = r_ref[:, 1] > r_ref[:, 0]
        np.testing.assert_array_equal(r_got[live], r_ref[live] + k0, err_msg=f"ranges, view {v}")
        assert np.all(r_got[~live, 0] == r_got[~live, 1]), f"empty tiles, view {v}"
        assert psnr(col[v], f.color) >= 50.0, v
        assert rel_l2(col[v], f.color) <= 1e-4, v
        g = f.state.backward(dpix[v])
        for k in ("means2D", "conic"):
            assert rel_l2(gv[k][v].cpu().numpy(), g[k]) <= 1e-4, (k, v, rel_l2(gv[k][v].cpu().numpy(), g[k]))
        g = {k: g[k].astype(np.float64) for k in ("means3D", "opacities", "scales", "rotations", "sh_dc", "sh_rest")}
        leaf_sum = g if leaf_sum is None else {k: leaf_sum[k] + g[k] for k in leaf_sum}
        k0 += kv
        seen += int(kv > 0)
    assert K == k0 and seen >= 6  # most views see the scene (the 90-degree yaw may not)
    for k, ref in leaf_sum.items():
        got = gv[k].cpu().numpy().reshape(ref.shape)
        assert rel_l2(got, ref) <= 1e-4, (k, rel_l2(got, ref))
