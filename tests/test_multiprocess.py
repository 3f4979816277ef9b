"""Multi-rank exchange on CPU (gloo, world size 2): the protocol of the multi-GPU path
(3d_gaussian_splatting_amd/bands.py, DESIGN.md §7, SURVEY §8e scaling version) with the CPU
oracle standing in for each rank's renderer (test infrastructure; on the GPU box the same
exchange moves the HIP path's 64-B splats over RCCL in bench.py).

Each rank owns a Gaussian shard and an instance-balanced band of tile rows:
* row histogram of its shard's instances -> all_reduce -> ``balance_bands`` (same cuts on every rank);
* for each band, the shard's Gaussians whose tile rect overlaps it, in shard order, go into
  that band's fixed-capacity block (header = count) -- the GPU path's block layout, here with
  the Gaussian's parameters as payload instead of its F1 record -- through
  ``bands.all_to_all_blocks``;
* the band owner renders its rows from the received Gaussians (ascending global id), the band
  images are all-gathered (``ImageGather``, bands padded to the tallest);
* each received Gaussian's band gradient goes back through ``all_to_all_blocks`` in the received
  slot layout, and the shard sums them per Gaussian in band order.

Checks (SURVEY §8e parity rules): the gathered image equals the single-process full render bit
for bit; the summed shard gradients equal the full render's leaf gradients within 1e-5
relative L2.
"""
import os
import socket
import tempfile

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import pkg, rel_l2

WORLD = 2
W, H = 96, 72  # 6 x 5 tiles
D = 2
LEAVES = ("means3D", "opacities", "scales", "rotations", "sh_dc", "sh_rest")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _scene():
    gr, sc = pkg("graphics"), pkg("scene")
    cam = gr.synthetic_camera(W, H)
    scene = sc.make_scene(cam, 400, max_sh_degree=D, seed=3)
    dpix = sc.make_dL_dpix(cam, seed=4)
    return cam, scene, dpix


def _params(scene, idx):
    """(n, F) f32 rows: the Gaussians' parameters (the stand-in splat payload)."""
    n = len(idx)
    return np.concatenate([scene.means3D[idx], scene.opacities[idx].reshape(n, 1), scene.scales[idx],
                           scene.rotations[idx], scene.sh_dc[idx].reshape(n, -1), scene.sh_rest[idx].reshape(n, -1)],
                          axis=1).astype(np.float32)


def _unparams(rows, M):
    n = rows.shape[0]
    return dict(means3D=rows[:, 0:3], opacities=rows[:, 3], scales=rows[:, 4:7], rotations=rows[:, 7:11],
                sh_dc=rows[:, 11:14].reshape(n, 1, 3), sh_rest=rows[:, 14:].reshape(n, M, 3))


def _oracle(cam, p, tile_rows=None):
    import gsr_oracle  # test infrastructure: the per-rank stand-in renderer
    return gsr_oracle.forward(cam, p["means3D"], p["opacities"], p["scales"], p["rotations"], p["sh_dc"],
                              p["sh_rest"], sh_degree=D, tile_rows=tile_rows)


def _grad_rows(g, n):
    return np.concatenate([g["means3D"], g["opacities"].reshape(n, 1), g["scales"], g["rotations"],
                           g["sh_dc"].reshape(n, -1), g["sh_rest"].reshape(n, -1)], axis=1).astype(np.float32)


def _worker(rank, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        bands = pkg("bands")
        cam, scene, dpix = _scene()
        P, gy = scene.P, cam.grid[1]
        M = scene.sh_rest.shape[1]
        g0, g1 = bands.gaussian_shard(P, WORLD, rank)
        mine = _params(scene, np.arange(g0, g1))
        shard = _unparams(mine, M)
        # per-tile-row instance histogram of this shard, summed over ranks -> balanced cuts
        hist = torch.tensor([int(_oracle(cam, shard, (y, y + 1)).num_rendered) for y in range(gy)], dtype=torch.int64)
        dist.all_reduce(hist)
        rows = bands.balance_bands(hist.numpy(), WORLD)
        band = (rows[rank], rows[rank + 1])
        # pack: per band the overlapping Gaussians in shard order, fixed-capacity blocks
        cap = g1 - g0
        F = mine.shape[1] + 1
        send = np.zeros((WORLD, 1 + cap, F), np.float32)
        sent = []
        for b in range(WORLD):
            tt = _oracle(cam, shard, (rows[b], rows[b + 1])).state.preprocess()["tiles_touched"]
            idx = np.nonzero(tt)[0]
            sent.append(idx)
            send[b, 0, 0] = len(idx)
            send[b, 1:1 + len(idx), 0] = (g0 + idx).astype(np.float32)  # global id (exact below 2^24)
            send[b, 1:1 + len(idx), 1:] = mine[idx]
        recv = bands.all_to_all_blocks(torch.from_numpy(send).reshape(-1), WORLD, dist).reshape(WORLD, 1 + cap, F)
        recv = recv.numpy()
        counts = [int(recv[s, 0, 0]) for s in range(WORLD)]
        got = np.concatenate([recv[s, 1:1 + counts[s]] for s in range(WORLD)])
        gid = got[:, 0].astype(np.int64)
        assert np.all(np.diff(gid) > 0), "splats must reach the band in ascending global id"
        f = _oracle(cam, _unparams(np.ascontiguousarray(got[:, 1:]), M), band)
        # the overflow words ride in the gather's footer row: every rank receives every rank's
        words = torch.tensor([counts[s] for s in range(WORLD)] + [1000 + rank, -1], dtype=torch.int32)
        img = bands.ImageGather(torch.from_numpy(f.color), rows, rank, dist, status=words)
        # backward: the band's gradient of every received Gaussian, back in the received slot layout
        gb = _grad_rows(f.state.backward(dpix), len(gid))
        G = gb.shape[1]
        back = np.zeros((WORLD, cap, G), np.float32)
        off = 0
        for s in range(WORLD):
            back[s, :counts[s]] = gb[off:off + counts[s]]
            off += counts[s]
        ret = bands.all_to_all_blocks(torch.from_numpy(back).reshape(-1), WORLD, dist).reshape(WORLD, cap, G).numpy()
        acc = np.zeros((g1 - g0, G), np.float32)
        for b in range(WORLD):  # band order: deterministic
            acc[sent[b]] += ret[b, :len(sent[b])]
        full = img.wait()
        allw = img.statuses()
        assert allw.dtype == torch.int32 and tuple(allw.shape) == (WORLD, WORLD + 2)
        assert allw[rank].tolist() == words.tolist()
        assert [int(allw[r, WORLD]) for r in range(WORLD)] == [1000 + r for r in range(WORLD)]
        assert all(int(allw[r, WORLD + 1]) == -1 for r in range(WORLD))  # bit-exact through the f32 slots
        parts = [torch.zeros((-(-P // WORLD), G)) for _ in range(WORLD)]
        pad = torch.zeros((-(-P // WORLD), G))
        pad[: g1 - g0] = torch.from_numpy(acc)
        dist.all_gather(parts, pad)
        if rank == 0:
            grads = torch.cat(parts)[:P].numpy()
            np.savez(os.path.join(outdir, "r0.npz"), image=full.numpy(), grads=grads, rows=np.array(rows))
    finally:
        dist.destroy_process_group()


def test_band_cuts():
    bands = pkg("bands")
    for gy in (1, 5, 68, 135):
        for world in range(1, min(gy, 8) + 1):
            rows = bands.equal_bands(gy, world)
            assert rows[0] == 0 and rows[-1] == gy and all(b > a for a, b in zip(rows, rows[1:]))
            rng = np.random.default_rng(gy * 10 + world)
            for counts in (rng.integers(0, 1000, gy), np.zeros(gy, np.int64), np.r_[np.zeros(gy - 1), [5]]):
                rows = bands.balance_bands(counts, world)
                assert rows[0] == 0 and rows[-1] == gy and all(b > a for a, b in zip(rows, rows[1:]))
    # a skewed histogram: the dense rows end up split across more bands
    counts = np.r_[np.full(10, 1000), np.full(58, 10)]
    rows = bands.balance_bands(counts, 4)
    loads = [counts[a:b].sum() for a, b in zip(rows, rows[1:])]
    assert max(loads) < 0.5 * counts.sum() and rows[1] < 10
    assert bands.gaussian_shard(10, 4, 3) == (9, 10) and bands.gaussian_shard(10, 4, 0) == (0, 3)


def test_gloo_two_ranks_match_single_process(oracle):
    port = _free_port()
    with tempfile.TemporaryDirectory() as outdir:
        mp.start_processes(_worker, args=(port, outdir), nprocs=WORLD, join=True, start_method="spawn")
        got = np.load(os.path.join(outdir, "r0.npz"))
        cam, scene, dpix = _scene()
        full = {k: v for k, v in zip(LEAVES, [scene.means3D, scene.opacities, scene.scales, scene.rotations,
                                               scene.sh_dc, scene.sh_rest])}
        f = _oracle(cam, full)
        g = f.state.backward(dpix)
        np.testing.assert_array_equal(got["image"], f.color)
        want = _grad_rows(g, scene.P)
        assert rel_l2(got["grads"], want) < 1e-5
        assert got["rows"][1] not in (0, cam.grid[1])


def test_overflow_ranks_word():
    """bands.overflow_ranks: the device agreement word counts the ranks whose counts exceed their
    own pair_cap / capacity (u32 counts, each rank against its own capacities)."""
    bands = pkg("bands")
    # (world 3, nb 3): counts..., band K, pair_cap, capacity
    w = torch.tensor([[10, 20, 30, 500, 32, 512],
                      [10, 40, 30, 500, 32, 512],    # a splat count past pair_cap
                      [1, 2, 3, 600, 32, 512]], dtype=torch.int32)  # band K past capacity
    g = bands.overflow_ranks(w)
    assert g.dtype == torch.int32 and g.shape == (1,) and int(g) == 2
    ok = torch.tensor([[32, 0, 1, 512, 32, 512]], dtype=torch.int32)
    assert int(bands.overflow_ranks(ok)) == 0
    huge = torch.tensor([[-1, 0, 0, 0, 32, 512]], dtype=torch.int32)  # 0xFFFFFFFF as u32
    assert int(bands.overflow_ranks(huge)) == 1


def _rect_rows(rng, n, gy):
    miny = rng.integers(0, gy, n)
    maxy = np.minimum(miny + 1 + rng.geometric(0.5, n) - 1, gy)  # exclusive, >= miny + 1
    return miny, maxy


def test_plan_from_stats_exact():
    """bands.plan_from_stats (the live re-plan of the multi-GPU step): the splat count of every
    (shard, band) pair for the cuts it picks equals a brute-force count over the rects, the band
    instance counts are the row sums, and the cuts are balance_bands of the instance histogram.
    The C++ gsr::plan_from_stats (through the extension's binding) agrees exactly."""
    bands = pkg("bands")
    rng = np.random.default_rng(7)
    for gy, world in ((68, 8), (30, 2), (5, 3), (135, 4)):
        shards = []
        inst = np.zeros(gy, np.int64)
        for s in range(world):
            miny, maxy = _rect_rows(rng, int(rng.integers(0, 3000)), gy)
            wd = rng.integers(1, 6, miny.size)
            for a, b_, w in zip(miny, maxy, wd):
                inst[a:b_] += w
            starts = np.bincount(miny, minlength=gy)
            ends = np.bincount(maxy - 1, minlength=gy)
            shards.append((miny, maxy, starts, ends))
        rows, max_splats, band_k = bands.plan_from_stats(inst, [x[2] for x in shards], [x[3] for x in shards], world)
        assert rows == bands.balance_bands(inst, world)
        assert band_k == [int(inst[rows[b]:rows[b + 1]].sum()) for b in range(world)]
        brute = max(int(((miny < rows[b + 1]) & (maxy > rows[b])).sum())
                    for miny, maxy, _, _ in shards for b in range(world))
        assert max_splats == brute
        try:
            ext = pkg("native").load_torch_ext()
        except Exception as e:  # pragma: no cover - the extension is built by __graft_entry__.build()
            import pytest
            pytest.skip(f"torch extension not loadable here: {e}")
        c_rows, c_max, c_k = ext.plan_from_stats([int(v) for v in inst], [[int(v) for v in x[2]] for x in shards],
                                                 [[int(v) for v in x[3]] for x in shards], world)
        assert list(c_rows) == rows and c_max == max_splats and list(c_k) == band_k
