"""GPU: the multi-GPU exchange code paths on the RCCL backend, with a single-rank process
group (the box has one GPU; the N-rank exchange arithmetic is covered by the gloo tests in
test_multiprocess.py).  Exercises the asynchronous count exchange (side stream, pinned host
copy, event) and the device all_to_all of GradExchange, and ImageGather's
all_gather_into_tensor."""
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


def test_grad_exchange_rccl(nccl):
    bands = pkg("bands")
    P = 5000
    g = torch.Generator(device="cpu").manual_seed(3)
    grad2d = torch.randn((P, 12), generator=g).cuda()
    cand = torch.nonzero(torch.rand(P, generator=g) < 0.3).flatten().to(torch.int32).cuda()
    xg = bands.GradExchange(cand, P, nccl)
    grad2d[:, 0] += 1.0  # produced after the exchange was planned, as B1's output is
    out = xg.run(grad2d)
    want = torch.zeros_like(grad2d)
    want[cand.long()] = grad2d[cand.long()]
    want[:, 9] = 0.0
    assert torch.equal(out, want)


def test_image_gather_rccl(nccl):
    bands = pkg("bands")
    gy, H, W = 5, 70, 48
    color = torch.rand((3, H, W)).cuda()
    img = bands.ImageGather(color, (0, gy), gy, nccl).wait()
    assert torch.equal(img, color)
