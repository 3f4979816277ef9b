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

``ImageGather`` starts the image all-gather asynchronously so it overlaps the blend backward.

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
