"""Known-answer tests restated from the reference's own Boost.Test cases.

They pin the INPUTS the rasterizer consumes: rotation / scaling-rotation / strip order /
covariance (src/utils/general_utils.cpp:147-292, src/scene/gaussian_model.cpp:409-453,496-562)
and the camera matrices (src/utils/graphics_utils.cpp:76-135).  Values are restated, not
copied; each test names the reference case it mirrors.  Checked against both the package's
host math and the CPU oracle's restatement.
"""
import math

import numpy as np
import pytest
import torch

from conftest import pkg

Q_ROT = [[0.5, 0.5, 0.5, 0.5], [0.25, 0.25, 0.25, 0.25]]
R_EXPECTED = np.array([[0, 0, 1], [1, 0, 0], [0, 1, 0]], np.float64)


def test_build_rotation_kat():  # general_utils.cpp:147-187
    general = pkg("general")
    R = general.build_rotation(torch.tensor(Q_ROT, dtype=torch.float64))
    for i in range(2):
        np.testing.assert_allclose(R[i].numpy(), R_EXPECTED, atol=1e-12)


def test_build_rotation_kat_oracle(oracle):
    for q in Q_ROT:
        np.testing.assert_allclose(oracle.build_rotation(q), R_EXPECTED, atol=1e-6)


@pytest.mark.parametrize("s", [0.5, 0.25])
def test_build_scaling_rotation_kat(s):  # general_utils.cpp:189-241
    general = pkg("general")
    L = general.build_scaling_rotation(torch.full((2, 3), s, dtype=torch.float64),
                                       torch.tensor(Q_ROT, dtype=torch.float64))
    np.testing.assert_allclose(L[0].numpy(), R_EXPECTED * s, atol=1e-12)


def test_strip_lowerdiag_order():  # general_utils.cpp:243-292: indices [0,1,2,4,5,8]
    general = pkg("general")
    M = torch.arange(9, dtype=torch.float64).reshape(1, 3, 3)
    np.testing.assert_array_equal(general.strip_symmetric(M)[0].numpy(), [0, 1, 2, 4, 5, 8])


@pytest.mark.parametrize("s,expect", [(0.5, 0.25), (0.25, 0.0625)])
def test_covariance_kat(s, expect, oracle):  # gaussian_model.cpp:409-453
    general = pkg("general")
    cov = general.build_covariance_from_scaling_rotation(
        torch.full((1, 3), s, dtype=torch.float64), 1.0, torch.tensor([Q_ROT[0]], dtype=torch.float64))
    np.testing.assert_allclose(cov[0].numpy(), [expect, 0, 0, expect, 0, expect], atol=1e-12)
    np.testing.assert_allclose(oracle.covariance([s] * 3, 1.0, Q_ROT[0]), [expect, 0, 0, expect, 0, expect],
                               atol=1e-7)


def test_covariance_raw_identity(oracle):  # gaussian_model.cpp:552-562: raw scale 0, raw rot ones
    general = pkg("general")
    s = torch.exp(torch.zeros(1, 3, dtype=torch.float64))
    cov = general.build_covariance_from_scaling_rotation(s, 1.0, torch.ones(1, 4, dtype=torch.float64))
    np.testing.assert_allclose(cov[0].numpy(), [1, 0, 0, 1, 0, 1], atol=1e-12)
    np.testing.assert_allclose(oracle.covariance([1, 1, 1], 1.0, [1, 1, 1, 1]), [1, 0, 0, 1, 0, 1], atol=1e-6)


def test_activations_kat():  # gaussian_model.cpp:496-550
    assert float(torch.nn.functional.normalize(torch.ones(1, 4), dim=1)[0, 0]) == pytest.approx(0.5)
    assert float(torch.sigmoid(torch.zeros(1))) == pytest.approx(0.5)
    assert float(torch.exp(torch.zeros(1))) == pytest.approx(1.0)


def test_projection_matrix_kat():  # graphics_utils.cpp:120-135
    gr = pkg("graphics")
    P = gr.get_projection_matrix(1.0, 10.0, math.pi / 2, math.pi / 2)
    assert P[0, 0] == pytest.approx(1.0, rel=1e-6)
    assert P[1, 1] == pytest.approx(1.0, rel=1e-6)
    assert P[0, 2] == 0.0 and P[1, 2] == 0.0
    assert P[3, 2] == 1.0
    assert P[2, 2] == pytest.approx(10.0 / 9, rel=1e-6)
    assert P[2, 3] == pytest.approx(-10.0 / 9, rel=1e-6)


def test_world2view_kat():  # graphics_utils.cpp:81-98
    gr = pkg("graphics")
    R = np.array([[1, 2, 0], [0, 1, 2], [0, 0, 1]], np.float64)
    Rt = gr.get_world2view(R, np.array([1.0, 2.0, 3.0]))
    assert Rt[0, 0] == Rt[1, 1] == Rt[2, 2] == Rt[3, 3] == 1.0
    assert Rt[0, 3] == 1.0 and Rt[1, 0] == 2.0 and Rt[1, 3] == 2.0 and Rt[2, 1] == 2.0 and Rt[2, 3] == 3.0


def test_world2view_2_kat():  # graphics_utils.cpp:100-118
    gr = pkg("graphics")
    R = np.array([[1, 2, 0], [0, 1, 2], [0, 0, 1]], np.float64)
    Rt = gr.get_world2view_2(R, np.array([1.0, 2.0, 3.0]), np.array([1.0, 1.0, 1.0]), 1.0)
    assert Rt[0, 0] == pytest.approx(1.0) and Rt[1, 1] == pytest.approx(1.0)
    assert Rt[2, 2] == pytest.approx(1.0) and Rt[3, 3] == pytest.approx(1.0)
    assert Rt[1, 0] == pytest.approx(2.0) and Rt[1, 3] == pytest.approx(-1.0)
    assert Rt[2, 1] == pytest.approx(2.0)


def test_camera_conventions():
    """camera.cpp:66-71: world_view = world2view_2^T (row-vector convention); the kernel's
    column-major read m[12..14] is the translation; campos = inv(world_view)[3,:3]."""
    gr = pkg("graphics")
    cam = gr.make_camera(np.eye(3), np.array([0.5, -1.0, 2.0]), math.radians(60), math.radians(40), 64, 48)
    V = cam.viewmatrix
    assert V[12] == pytest.approx(0.5) and V[13] == pytest.approx(-1.0) and V[14] == pytest.approx(2.0)
    np.testing.assert_allclose(cam.campos, [-0.5, 1.0, -2.0], atol=1e-6)
    assert cam.tanfovx == pytest.approx(math.tan(math.radians(30)), rel=1e-6)
