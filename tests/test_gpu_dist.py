"""GPU: the multi-GPU path (bands.ShardStep: Gaussian shard F1 -> splat all-to-all -> band
F2..F6 -> image all-gather -> band B1 -> gradient all-to-all -> shard B2) on the RCCL backend
with a single-rank process group (the box has one GPU; the N-rank exchange protocol is covered
by the gloo test in test_multiprocess.py and the N-rank compute by test_gpu_parity's
one-process rank simulation).  With one rank the step must reproduce the single-GPU
forward + backward bit for bit."""
import os
import socket

import pytest
import torch

from conftest import pkg

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def nccl():
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    yield dist
    dist.destroy_process_group()


def test_shard_step_rccl_single_rank(nccl):
    bands, R, gr, sc = pkg("bands"), pkg("rasterizer"), pkg("graphics"), pkg("scene")
    dev = torch.device("cuda", 0)
    cam = gr.synthetic_camera(320, 240)
    s = sc.make_scene(cam, 20000, max_sh_degree=3, seed=21)
    t = lambda a: torch.tensor(a, device=dev)
    inputs = dict(means3D=t(s.means3D), opacities=t(s.opacities), scales=t(s.scales), rotations=t(s.rotations),
                  sh_dc=t(s.sh_dc), sh_rest=t(s.sh_rest))
    dpix = t(sc.make_dL_dpix(cam, seed=22))
    step = bands.ShardStep(R.ShardRasterizer(dev), cam, inputs, 3, nccl).plan()
    img, g, sh, st = step.step(dpix)
    rast = R.CAbiRasterizer(dev)
    full = rast.forward(cam, **inputs, sh_degree=3)
    gf = rast.backward(full, dpix)
    assert torch.equal(img, full.color)
    assert st.num_rendered == full.num_rendered
    assert torch.equal(sh.radii, full.radii)
    for k, v in g.items():
        assert torch.equal(v, gf[k]), k


def test_image_gather_rccl(nccl):
    bands = pkg("bands")
    gy, H, W = 5, 70, 48
    color = torch.rand((3, H, W)).cuda()
    img = bands.ImageGather(color, [0, gy], 0, nccl).wait()
    assert torch.equal(img, color)
