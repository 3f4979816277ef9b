"""GPU: batched multi-view forward (gsr_forward_batch).

A batch must give, view by view, exactly what gsr_forward gives for that camera alone --
colour, radii, instance count, the sorted (tile, gid) list and tile ranges bit for bit -- and
each view's buffers must drive gsr_backward to the same gradients bit for bit (the batch only
changes when the host waits, not what any kernel computes).
"""
import math

import numpy as np
import pytest
import torch

from conftest import pkg

pytestmark = pytest.mark.gpu


def _rot_y(deg):
    a = math.radians(deg)
    return np.array([[math.cos(a), 0, math.sin(a)], [0, 1, 0], [-math.sin(a), 0, math.cos(a)]])


def _cams():
    gr = pkg("graphics")
    out = []
    for deg, (w, h), t in [(0, (320, 240), (0, 0, 0)), (8, (320, 240), (0.3, 0, 0)), (-12, (256, 192), (0, 0.2, 0.5)),
                           (4, (200, 160), (0, 0, -0.5)), (90, (128, 96), (0, 0, 0))]:  # last: looks away (K ~ 0)
        fx = math.radians(60.0)
        fy = 2 * math.atan(math.tan(fx / 2) * h / w)
        out.append(gr.make_camera(_rot_y(deg), np.array(t, float), fx, fy, w, h))
    return out


def _scene():
    gr, sc = pkg("graphics"), pkg("scene")
    s = sc.make_scene(gr.synthetic_camera(320, 240), 20000, max_sh_degree=3, seed=21)
    return (s.means3D, s.opacities, s.scales, s.rotations, s.sh_dc, s.sh_rest)


def test_batch_equals_single_views():
    R, native = pkg("rasterizer"), pkg("native")
    rast = R.CAbiRasterizer("cuda")
    cams = _cams()
    args = _scene()
    batch = rast.forward_batch(cams, *args, sh_degree=3, bg=(0.1, 0.2, 0.3))
    assert len(batch) == len(cams)
    for cam, b in zip(cams, batch):
        a = rast.forward(cam, *args, sh_degree=3, bg=(0.1, 0.2, 0.3))
        assert torch.equal(a.color, b.color)
        assert torch.equal(a.radii, b.radii)
        assert a.num_rendered == b.num_rendered
        K = a.num_rendered
        if K:
            for what in (native.VIEW_SORTED_GID, native.VIEW_SORTED_TILE):
                assert torch.equal(a.view(what, torch.int32, K), b.view(what, torch.int32, K))
        tiles = cam.grid[0] * cam.grid[1]
        assert torch.equal(a.view(native.VIEW_RANGES, torch.int32, 2 * tiles),
                           b.view(native.VIEW_RANGES, torch.int32, 2 * tiles))
        dpix = torch.rand((3, cam.height, cam.width), device="cuda", generator=torch.Generator("cuda").manual_seed(3))
        ga, gb = rast.backward(a, dpix), rast.backward(b, dpix)
        for k in ga:
            assert torch.equal(ga[k], gb[k]), k
    assert batch[-1].num_rendered < batch[0].num_rendered  # the camera looking away sees little


def test_batch_limits():
    R = pkg("rasterizer")
    rast = R.CAbiRasterizer("cuda")
    args = _scene()
    assert rast.forward_batch([], *args, sh_degree=3) == []
    cam = _cams()[0]
    with pytest.raises(RuntimeError, match="views"):
        rast.forward_batch([cam] * 65, *args, sh_degree=3)
    one = rast.forward_batch([cam], *args, sh_degree=3)[0]
    assert torch.equal(one.color, rast.forward(cam, *args, sh_degree=3).color)
    empty = rast.forward_batch([cam, cam], np.zeros((0, 3)), np.zeros(0), np.zeros((0, 3)), np.zeros((0, 4)),
                               np.zeros((0, 1, 3)), None, sh_degree=0, bg=(1, 1, 1))
    assert all(float(e.color.min()) == 1.0 for e in empty)
