"""Screen-space tile-row bands: the multi-GPU partition of the rasterizer (DESIGN.md §7,
SURVEY §8e).

Rank r of N owns tile rows [rows[r], rows[r+1]) with rows[i] = floor(i * grid_y / N).  It
bins and blends only those rows (``gsr_raster_settings.tile_y0/y1``), so its image band is
bit-identical to the same rows of a single-GPU render.  The exchange is two collectives:

* ``gather_image``: all-gather of the bands (padded to the tallest band) into the full
  (3, H, W) image;
* ``reduce_grad2d``: sum over ranks of the per-Gaussian 2D gradients (grad2d, P x 12
  floats) that ``gsr_backward_blend`` leaves for each band; B2 then runs on the sum; or
  ``reduce_scatter_grad2d``: each rank receives the sum for its own Gaussian slice
  (``gaussian_slice``) and runs B2 on that slice only (``gsr_backward_preprocess_range``),
  so the leaf gradients -- and an optimizer step after them -- are sharded by Gaussian.

``exchange_grad2d`` is the sparse form of the reduce-scatter: only a band's candidate
Gaussians carry gradient, so only their rows travel.  ``ImageGather`` starts the image
all-gather asynchronously so it overlaps the blend backward.

Both work on any torch.distributed backend (RCCL on the GPU box, gloo in the CPU tests).
"""
from __future__ import annotations

import torch

TILE = 16


def band_rows(grid_y: int, world: int, rank: int) -> tuple[int, int]:
    """Tile-row range [y0, y1) of `rank` among `world` contiguous bands."""
    return (rank * grid_y) // world, ((rank + 1) * grid_y) // world


def band_pixel_rows(band: tuple[int, int], height: int) -> tuple[int, int]:
    """Pixel-row range [py0, py1) covered by a tile-row band, clipped to the image."""
    return min(band[0] * TILE, height), min(band[1] * TILE, height)


def max_band_pixel_rows(grid_y: int, world: int) -> int:
    return max(b - a for a, b in (band_rows(grid_y, world, r) for r in range(world))) * TILE


def gaussian_slice(P: int, world: int, rank: int) -> tuple[int, int]:
    """Gaussians [g0, g1) whose leaf gradients rank `rank` owns (equal slices of
    ceil(P / world), the last one short)."""
    S = -(-P // world)
    return min(rank * S, P), min((rank + 1) * S, P)


def padded_rows(P: int, world: int) -> int:
    return -(-P // world) * world


def reduce_scatter_grad2d(grad2d_padded: torch.Tensor, dist, group=None) -> torch.Tensor:
    """Sum grad2d (padded_rows(P, world) x 12) over ranks; return this rank's slice
    (ceil(P / world) rows, the tail beyond P is padding)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    S = grad2d_padded.shape[0] // world
    if dist.get_backend(group) == "gloo":  # no reduce_scatter in gloo: all-reduce, keep the slice
        dist.all_reduce(grad2d_padded, group=group)
        return grad2d_padded[rank * S:(rank + 1) * S]
    out = grad2d_padded.new_empty((S,) + tuple(grad2d_padded.shape[1:]))
    dist.reduce_scatter_tensor(out, grad2d_padded, group=group)
    return out


def exchange_grad2d(grad2d: torch.Tensor, cand: torch.Tensor, P: int, dist, group=None) -> torch.Tensor:
    """Sparse reduce-scatter of the 2D gradients: a band only produced rows for its candidate
    Gaussians (``cand``: their ids, e.g. ``GSR_VIEW_GID_BY_RANK``), so each rank sends just
    those rows, bucketed by owning rank (``gaussian_slice``), in one all_to_all.  The owner
    places every received row in a per-source dense slab and sums the slabs, so the result
    is the same fixed-order sum whatever the arrival order.  Returns this rank's slice
    (ceil(P / world) rows x 12).  The gid rides in padding column 9 of each row."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    S = -(-P // world)
    width = grad2d.shape[1]
    if width < 10:
        raise ValueError("exchange_grad2d: rows need a padding column 9 (GSR_GRAD2D_STRIDE = 12)")
    dev = grad2d.device
    cand = cand.to(torch.int64)
    owner = torch.div(cand, S, rounding_mode="floor")
    order = torch.argsort(owner, stable=True)
    cs = cand[order]
    rows = grad2d.index_select(0, cs)
    rows[:, 9] = cs.to(torch.int32).view(torch.float32)
    send = torch.bincount(owner, minlength=world)
    # gloo has no device all-to-all: stage through host memory there
    host = dist.get_backend(group) == "gloo" and dev.type != "cpu"
    xdev = torch.device("cpu") if host else dev
    send_x = send.to(xdev)
    recv_x = torch.empty_like(send_x)
    dist.all_to_all_single(recv_x, send_x, group=group)
    sc, rc = send_x.tolist(), recv_x.tolist()
    got = torch.empty((sum(rc), width), dtype=rows.dtype, device=xdev)
    dist.all_to_all_single(got, rows.to(xdev), rc, sc, group=group)
    got = got.to(dev)
    gid = got[:, 9].contiguous().view(torch.int32).to(torch.int64) - rank * S
    src = torch.repeat_interleave(torch.arange(world, device=dev), torch.tensor(rc, device=dev))
    dense = grad2d.new_zeros((world, S, width))
    dense[src, gid] = got
    out = dense.sum(0)
    out[:, 9] = 0.0
    return out


class ImageGather:
    """Asynchronous all-gather of the band images: start it after the forward, wait() for the
    full (3, H, W) image after the backward -- the collective runs on the communicator's own
    stream while the blend backward runs on the compute stream."""

    def __init__(self, color: torch.Tensor, band: tuple[int, int], grid_y: int, dist, group=None):
        self.world = dist.get_world_size(group)
        _, self.H, W = color.shape
        self.grid_y = grid_y
        rows = max_band_pixel_rows(grid_y, self.world)
        py0, py1 = band_pixel_rows(band, self.H)
        self.mine = color.new_zeros((3, rows, W))
        self.mine[:, : py1 - py0] = color[:, py0:py1]
        self.buf = color.new_empty((self.world, 3, rows, W))
        if dist.get_backend(group) != "gloo":
            self.work = dist.all_gather_into_tensor(self.buf.view(-1), self.mine.view(-1), group=group,
                                                    async_op=True)
        else:
            self.work = dist.all_gather(list(self.buf.unbind(0)), self.mine, group=group, async_op=True)
        self.color = color

    def wait(self) -> torch.Tensor:
        self.work.wait()
        out = self.color.new_empty((3, self.H, self.color.shape[2]))
        for r in range(self.world):
            a0, a1 = band_pixel_rows(band_rows(self.grid_y, self.world, r), self.H)
            out[:, a0:a1] = self.buf[r, :, : a1 - a0]
        return out


def gather_image(color: torch.Tensor, band: tuple[int, int], grid_y: int, dist, group=None) -> torch.Tensor:
    """All-gather the band rows of `color` (3, H, W; only this rank's band is valid) into the
    full image (synchronous form of ImageGather).  Bands are padded to the tallest one so a
    single all_gather_into_tensor (one RCCL call) moves them."""
    return ImageGather(color, band, grid_y, dist, group).wait()


def reduce_grad2d(grad2d: torch.Tensor, dist, group=None, async_op: bool = False):
    """Sum the per-band 2D gradients over ranks in place (every rank gets the total)."""
    return dist.all_reduce(grad2d, group=group, async_op=async_op)
