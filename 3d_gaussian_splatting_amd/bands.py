"""Screen-space tile-row bands: the multi-GPU partition of the rasterizer (DESIGN.md §7,
SURVEY §8e).

Rank r of N owns tile rows [rows[r], rows[r+1]) with rows[i] = floor(i * grid_y / N).  It
bins and blends only those rows (``gsr_raster_settings.tile_y0/y1``), so its image band is
bit-identical to the same rows of a single-GPU render.  The exchange is two collectives:

* ``gather_image``: all-gather of the bands (padded to the tallest band) into the full
  (3, H, W) image;
* ``reduce_grad2d``: sum over ranks of the per-Gaussian 2D gradients (grad2d, P x 12
  floats) that ``gsr_backward_blend`` leaves for each band; B2 then runs on the sum.

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


def gather_image(color: torch.Tensor, band: tuple[int, int], grid_y: int, dist, group=None) -> torch.Tensor:
    """All-gather the band rows of `color` (3, H, W; only this rank's band is valid) into the
    full image.  Bands are padded to the tallest one so a single all_gather_into_tensor
    (one RCCL call) moves them."""
    world = dist.get_world_size(group)
    _, H, W = color.shape
    rows = max_band_pixel_rows(grid_y, world)
    py0, py1 = band_pixel_rows(band, H)
    mine = color.new_zeros((3, rows, W))
    mine[:, : py1 - py0] = color[:, py0:py1]
    buf = color.new_empty((world, 3, rows, W))
    if hasattr(dist, "all_gather_into_tensor") and dist.get_backend(group) != "gloo":
        dist.all_gather_into_tensor(buf.view(-1), mine.view(-1), group=group)
    else:
        dist.all_gather(list(buf.unbind(0)), mine, group=group)
    out = color.new_empty((3, H, W))
    for r in range(world):
        b = band_rows(grid_y, world, r)
        a0, a1 = band_pixel_rows(b, H)
        out[:, a0:a1] = buf[r, :, : a1 - a0]
    return out


def reduce_grad2d(grad2d: torch.Tensor, dist, group=None, async_op: bool = False):
    """Sum the per-band 2D gradients over ranks in place (every rank gets the total)."""
    return dist.all_reduce(grad2d, group=group, async_op=async_op)
