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

``GradExchange`` / ``exchange_grad2d`` is the sparse form of the reduce-scatter: only a
band's candidate Gaussians carry gradient, so only their rows travel.  ``ImageGather`` starts the image
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


_SIDE_STREAMS: dict = {}


def _side_stream(dev: torch.device) -> torch.cuda.Stream:
    if dev not in _SIDE_STREAMS:
        _SIDE_STREAMS[dev] = torch.cuda.Stream(dev)
    return _SIDE_STREAMS[dev]


class GradExchange:
    """Sparse reduce-scatter of the 2D gradients: a band only produced rows for its candidate
    Gaussians (``cand``: their ids, e.g. ``GSR_VIEW_GID_BY_RANK``), so each rank sends just
    those rows, bucketed by owning rank (``gaussian_slice``), in one all_to_all.  The gid
    rides in padding column 9 of each row.

    Two phases so the host never stalls the GPU: the constructor (right after the forward --
    the candidates are known then) starts the all_to_all of the per-owner row counts and
    copies the received counts to pinned host memory on a side stream that waits only for
    that collective; ``run(grad2d)`` (after the blend backward has been enqueued) reads the
    counts -- long since arrived -- and moves the rows.  The owner sums the rows it receives
    source by source in rank order (each source sends a Gaussian at most once, so every
    ``index_add_`` has unique indices): a fixed-order, deterministic sum.  ``run`` returns
    this rank's slice (ceil(P / world) rows x 12)."""

    def __init__(self, cand: torch.Tensor, P: int, dist, group=None):
        self.dist, self.group = dist, group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.S = -(-P // self.world)
        cand = cand.to(torch.int64)
        self.dev = cand.device
        owner = torch.div(cand, self.S, rounding_mode="floor")
        order = torch.argsort(owner, stable=True)
        self.cs = cand[order]
        send = torch.bincount(owner, minlength=self.world)
        # gloo has no device all-to-all: stage through host memory there
        self.host = dist.get_backend(group) == "gloo" and self.dev.type != "cpu"
        if self.host or self.dev.type == "cpu":
            xdev = torch.device("cpu")
            send_x = send.to(xdev)
            recv_x = torch.empty_like(send_x)
            dist.all_to_all_single(recv_x, send_x, group=group)
            self.sc, self.rc = send_x.tolist(), recv_x.tolist()
            self.event = None
            return
        recv = torch.empty_like(send)
        work = dist.all_to_all_single(recv, send, group=group, async_op=True)
        side = _side_stream(self.dev)
        side.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(side):
            work.wait()  # the side stream waits for the collective, the compute stream does not
            self.send_h = torch.empty(self.world, dtype=torch.int64, pin_memory=True)
            self.recv_h = torch.empty(self.world, dtype=torch.int64, pin_memory=True)
            self.send_h.copy_(send, non_blocking=True)
            self.recv_h.copy_(recv, non_blocking=True)
            self.event = torch.cuda.Event()
            self.event.record(side)
        self._keep = (send, recv)

    def run(self, grad2d: torch.Tensor) -> torch.Tensor:
        width = grad2d.shape[1]
        if width < 10:
            raise ValueError("GradExchange: rows need a padding column 9 (GSR_GRAD2D_STRIDE = 12)")
        if self.event is not None:
            self.event.synchronize()
            self.sc, self.rc = self.send_h.tolist(), self.recv_h.tolist()
        dev = grad2d.device
        rows = grad2d.index_select(0, self.cs)
        rows[:, 9] = self.cs.to(torch.int32).view(torch.float32)
        xdev = torch.device("cpu") if self.host else dev
        got = torch.empty((sum(self.rc), width), dtype=rows.dtype, device=xdev)
        self.dist.all_to_all_single(got, rows.to(xdev), self.rc, self.sc, group=self.group)
        got = got.to(dev)
        gid = got[:, 9].contiguous().view(torch.int32).to(torch.int64) - self.rank * self.S
        out = grad2d.new_zeros((self.S, width))
        off = 0
        for n in self.rc:  # source ranks in order
            if n:
                out.index_add_(0, gid[off:off + n], got[off:off + n])
            off += n
        out[:, 9] = 0.0
        return out


def exchange_grad2d(grad2d: torch.Tensor, cand: torch.Tensor, P: int, dist, group=None) -> torch.Tensor:
    """One-call form of ``GradExchange``: count exchange and row exchange back to back."""
    return GradExchange(cand, P, dist, group).run(grad2d)


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
