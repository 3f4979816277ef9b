"""Multi-rank band sharding on CPU (gloo, world size 2): the exchange code of
3d_gaussian_splatting_amd/bands.py with the CPU oracle standing in for each rank's renderer
(test infrastructure; the GPU path runs the same exchange over RCCL in bench.py).

Checks (SURVEY §8e parity rules):
* the all-gathered band images equal the single-process full render bit for bit;
* the reduce-scatter of the band-local 2D gradients (mean2D, conic, opacity, colour -- what
  gsr_backward_blend returns as grad2d) gives each rank its Gaussian slice of the full-image
  2D gradients (slices re-assembled here to compare), and the leaf gradients after the chain
  rule (B2 is linear in grad2d) sum to the full-image ones, within 1e-5 relative L2;
* bands partition the tile rows for every world size up to 8 and uneven heights.
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import pkg, rel_l2

WORLD = 2
W, H = 96, 72  # 6 x 5 tiles: uneven band split for 2 ranks (2 + 3 tile rows)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _scene():
    gr, sc = pkg("graphics"), pkg("scene")
    cam = gr.synthetic_camera(W, H)
    scene = sc.make_scene(cam, 400, max_sh_degree=2, seed=3)
    dpix = sc.make_dL_dpix(cam, seed=4)
    return cam, scene, dpix


def _render(cam, scene, dpix, tile_rows=None):
    import gsr_oracle  # test infrastructure: the per-rank stand-in renderer
    f = gsr_oracle.forward(cam, scene.means3D, scene.opacities, scene.scales, scene.rotations, scene.sh_dc,
                           scene.sh_rest, sh_degree=2, tile_rows=tile_rows)
    return f, f.state.backward(dpix)


def _worker(rank, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        bands = pkg("bands")
        cam, scene, dpix = _scene()
        gy = (H + 15) // 16
        band = bands.band_rows(gy, WORLD, rank)
        f, g = _render(cam, scene, dpix, tile_rows=band)
        img = bands.ImageGather(torch.from_numpy(f.color), band, gy, dist)
        P = g["means2D"].shape[0]
        g2d = np.concatenate([g["means2D"][:, :2], g["conic"], g["opacities"], g["colors"]], axis=1)
        padded = torch.zeros((bands.padded_rows(P, WORLD), 12))  # GSR_GRAD2D_STRIDE rows
        padded[:P, :9] = torch.from_numpy(g2d)
        g0, g1 = bands.gaussian_slice(P, WORLD, rank)
        mine = bands.reduce_scatter_grad2d(padded.clone(), dist)[: g1 - g0].clone()
        # sparse form: only the band's candidates (Gaussians with tiles in the band) travel
        cand = torch.from_numpy(np.nonzero(f.state.preprocess()["tiles_touched"])[0].astype(np.int32))
        sparse = bands.exchange_grad2d(padded[:P].clone(), cand, P, dist)[: g1 - g0]
        assert torch.equal(sparse[:, :9], mine[:, :9]) or float((sparse[:, :9] - mine[:, :9]).abs().max()) < 1e-6
        slices = [torch.zeros_like(padded[: padded.shape[0] // WORLD]) for _ in range(WORLD)]
        dist.all_gather(slices, torch.nn.functional.pad(mine, (0, 0, 0, slices[0].shape[0] - mine.shape[0])))
        grad2d = torch.cat(slices)[:P, :9]
        full = img.wait()
        leaf = {k: torch.from_numpy(g[k].copy()) for k in ("means3D", "scales", "rotations", "sh_dc", "sh_rest",
                                                          "opacities")}
        for v in leaf.values():
            dist.all_reduce(v)
        if rank == 0:
            np.savez(os.path.join(outdir, "r0.npz"), image=full.numpy(), grad2d=grad2d.numpy(),
                     **{f"leaf_{k}": v.numpy() for k, v in leaf.items()})
    finally:
        dist.destroy_process_group()


def test_band_rows_partition():
    bands = pkg("bands")
    for gy in (1, 5, 68, 135):
        for world in range(1, 9):
            rows = [bands.band_rows(gy, world, r) for r in range(world)]
            assert rows[0][0] == 0 and rows[-1][1] == gy
            assert all(rows[i][1] == rows[i + 1][0] for i in range(world - 1))
            assert bands.max_band_pixel_rows(gy, world) == max(b - a for a, b in rows) * 16


def test_gloo_two_ranks_match_single_process(oracle):
    port = _free_port()
    with tempfile.TemporaryDirectory() as outdir:
        mp.start_processes(_worker, args=(port, outdir), nprocs=WORLD, join=True, start_method="spawn")
        got = np.load(os.path.join(outdir, "r0.npz"))
        cam, scene, dpix = _scene()
        f, g = _render(cam, scene, dpix)
        np.testing.assert_array_equal(got["image"], f.color)
        want2d = np.concatenate([g["means2D"][:, :2], g["conic"], g["opacities"], g["colors"]], axis=1)
        assert rel_l2(got["grad2d"], want2d) < 1e-5
        for k in ("means3D", "scales", "rotations", "sh_dc", "sh_rest", "opacities"):
            assert rel_l2(got[f"leaf_{k}"], g[k]) < 1e-5, k
