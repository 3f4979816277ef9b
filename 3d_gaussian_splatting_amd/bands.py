"""Multi-GPU partition of the rasterizer (SURVEY §8e "scaling version").

Rank r of N owns

* the Gaussian shard [g0, g1) = ``gaussian_shard(P, N, r)`` (contiguous, in rank order): it
  runs F1 (preprocess) and B2 (preprocess backward) for those Gaussians only, and its leaf
  gradients -- and an optimizer step after them -- stay sharded;
* the band of tile rows [rows[r], rows[r+1]): it bins, blends (F2..F6) and runs the blend
  backward (B1) for those rows only.  ``balance_bands`` places the cuts so each band holds about
  the same number of (Gaussian, tile) instances, from the per-tile-row instance histogram the
  shard forward accumulates (``row_hist``, summed over ranks).

One step (``ShardStep.step``) moves data three times, all over torch.distributed (RCCL on the
GPU box, gloo in the CPU tests):

1. all-to-all of the projected Gaussians ("splats", 64 B): shard -> every band its tile rect
   overlaps.  Fixed-capacity blocks (``pair_cap`` splats per (source, band) pair, sized once
   from a probe step) so the sizes never have to reach the host: one ``all_to_all_single``
   with equal splits, the true counts ride in each block's header;
2. all-gather of the band images, padded to the tallest band, asynchronous: it overlaps B1;
3. all-to-all back of each splat's 48-B 2D gradient to its shard, which sums them per
   Gaussian in band order (deterministic) before B2.

Splats reach a band in (source rank, shard index) order, i.e. ascending global Gaussian id, so
the band's canonical (tile, depth, gid) order and every pixel equal the single-GPU render.
"""
from __future__ import annotations

import numpy as np
import torch

TILE = 16


def gaussian_shard(P: int, world: int, rank: int) -> tuple[int, int]:
    """Gaussians [g0, g1) rank `rank` owns (slices of ceil(P / world), the last one short)."""
    S = -(-P // world)
    return min(rank * S, P), min((rank + 1) * S, P)


def equal_bands(grid_y: int, world: int) -> list[int]:
    """Tile-row cuts of `world` bands of (nearly) equal height: rows[0] = 0 .. rows[world] = grid_y."""
    return [(r * grid_y) // world for r in range(world + 1)]


def balance_bands(row_counts, world: int) -> list[int]:
    """Tile-row cuts so each band holds about total / world instances (row_counts[y] = the
    instances in tile row y).  Each cut is the row boundary whose prefix sum is nearest the
    target k * total / world, kept strictly increasing so no band is empty (world <= rows)."""
    c = np.asarray(row_counts, dtype=np.float64)
    gy = len(c)
    if world > gy:
        raise ValueError(f"{world} bands need at least as many tile rows (got {gy})")
    pre = np.concatenate([[0.0], np.cumsum(c)])
    total = pre[-1]
    if total <= 0:
        return equal_bands(gy, world)
    rows = [0]
    for k in range(1, world):
        t = k * total / world
        y = int(np.argmin(np.abs(pre - t)))
        y = max(y, rows[-1] + 1)            # at least one row per band ...
        y = min(y, gy - (world - k))        # ... and room for the bands after it
        rows.append(y)
    rows.append(gy)
    return rows


def band_pixel_rows(band: tuple[int, int], height: int) -> tuple[int, int]:
    """Pixel-row range [py0, py1) covered by a tile-row band, clipped to the image."""
    return min(band[0] * TILE, height), min(band[1] * TILE, height)


def round_up(x: int, m: int = 256) -> int:
    return -(-int(x) // m) * m


def plan_from_stats(inst, starts, ends, world: int):
    """Band cuts from one step's row statistics (GSR_FLAG_ROW_SPANS): inst[y] = the instances in
    tile row y over all shards; starts[s][y] / ends[s][y] = shard s's visible Gaussians whose tile
    rect starts / ends (last row) in row y.  The splats shard s sends to band [r0, r1) are exactly
    sum_{y<r1} starts[s][y] - sum_{y<r0} ends[s][y] (a rect meets the band iff it starts before r1
    and does not end before r0), so the needed capacities follow for any cuts.
    -> (rows, max splats per (shard, band), instances per band).  gsr::plan_from_stats is the
    same arithmetic in C++."""
    inst = np.asarray(inst, np.int64)
    rows = balance_bands(inst, world)
    band_k = [int(inst[rows[b]:rows[b + 1]].sum()) for b in range(world)]
    max_splats = 0
    for s_, e_ in zip(starts, ends):
        ps = np.concatenate([[0], np.cumsum(np.asarray(s_, np.int64))])
        pe = np.concatenate([[0], np.cumsum(np.asarray(e_, np.int64))])
        max_splats = max(max_splats, max(int(ps[rows[b + 1]] - pe[rows[b]]) for b in range(world)))
    return rows, max_splats, band_k


class ImageGather:
    """Asynchronous all-gather of the band images: start it after the band forward, wait() for
    the full (3, H, W) image after the backward -- the collective runs on the communicator's
    own stream while the blend backward runs on the compute stream.  Bands are padded to the
    tallest one so a single all_gather_into_tensor (one RCCL call) moves them."""

    def __init__(self, color: torch.Tensor, rows: list, rank: int, dist, group=None, status=None):
        """status: an optional int32 device tensor (this rank's overflow words) that rides in a
        footer row of the gathered bands, so that every rank sees every rank's words."""
        self.world = len(rows) - 1
        _, self.H, W = color.shape
        self.rows = rows
        tall = max(band_pixel_rows((rows[r], rows[r + 1]), self.H)[1] - band_pixel_rows((rows[r], rows[r + 1]),
                                                                                     self.H)[0]
                   for r in range(self.world))
        py0, py1 = band_pixel_rows((rows[rank], rows[rank + 1]), self.H)
        self.tall = max(tall, 1)
        self.S = 0 if status is None else int(status.numel())
        if self.S > W:
            raise ValueError(f"{self.S} status words do not fit a {W}-pixel footer row")
        foot = 1 if self.S else 0
        self.mine = color.new_zeros((3, self.tall + foot, W))
        self.mine[:, : py1 - py0] = color[:, py0:py1]
        if self.S:  # the words' bits in f32 slots (a view, no conversion)
            self.mine[0, self.tall, : self.S].view(torch.int32).copy_(status.reshape(-1).to(torch.int32))
        self.buf = color.new_empty((self.world, 3, self.tall + foot, W))
        if dist.get_backend(group) != "gloo":
            self.work = dist.all_gather_into_tensor(self.buf.view(-1), self.mine.view(-1), group=group,
                                                    async_op=True)
        else:
            self.work = dist.all_gather(list(self.buf.unbind(0)), self.mine, group=group, async_op=True)
        self.color = color

    def statuses(self) -> torch.Tensor:
        """(world, S) int32 device tensor: every rank's status words (after wait())."""
        return self.buf[:, 0, self.tall, : self.S].contiguous().view(torch.int32)

    def wait(self) -> torch.Tensor:
        self.work.wait()
        out = self.color.new_empty((3, self.H, self.color.shape[2]))
        for r in range(self.world):
            a0, a1 = band_pixel_rows((self.rows[r], self.rows[r + 1]), self.H)
            out[:, a0:a1] = self.buf[r, :, : a1 - a0]
        return out


def all_to_all_blocks(send: torch.Tensor, world: int, dist, group=None) -> torch.Tensor:
    """Equal-split all-to-all of `world` contiguous blocks (block b -> rank b).  gloo has no
    device all-to-all: staged through host memory there."""
    recv = torch.empty_like(send)
    if dist.get_backend(group) == "gloo" and send.device.type != "cpu":
        h = send.cpu()
        hr = torch.empty_like(h)
        dist.all_to_all_single(hr, h, group=group)
        recv.copy_(hr)
    else:
        dist.all_to_all_single(recv, send, group=group)
    return recv


class ShardOverflowError(RuntimeError):
    """A step's splats or band instances exceeded the capacities ``plan`` sized: that step's
    render was truncated (the kernels drop what does not fit and stay inside their buffers).
    ``step`` is the index of the offending step, ``counts`` the per-band splat counts that
    rank packed (against ``pair_cap``) and ``band_k`` its band's instance count (against
    ``capacity``).  Re-plan (``ShardStep.plan``) and re-run from that step."""

    def __init__(self, step: int, counts, pair_cap: int, band_k: int, capacity: int, rank=None):
        self.step, self.counts, self.pair_cap = step, list(counts), pair_cap
        self.band_k, self.capacity, self.rank = band_k, capacity, rank
        who = "" if rank is None else f" on rank {rank}"
        super().__init__(f"multi-GPU step {step} overflowed{who}: splats per band {self.counts} vs pair_cap "
                         f"{pair_cap}, band instances {band_k} vs capacity {capacity}")


def overflow_ranks(words: torch.Tensor, nb: int | None = None) -> torch.Tensor:
    """Device-side agreement word: the number of ranks whose step overflowed, as a (1,) int32
    tensor on the words' device, computed without a host wait.  `words`: (world, nb + 3) int32,
    every rank's per-band splat counts, band K, pair_cap and capacity (the gathered footer;
    `nb` = the number of counts when row statistics follow, else (words.shape[1] - 3)).
    Every rank computes it from the same gathered words, so every rank holds the same value: a
    training loop passes it as the guard of its optimizer step (``gsr_adam_step_guarded`` /
    ``gsr_densify_stats_guarded`` with guard_cap = 0, trainer.adam_step(guard=(word, 0))) so that
    a truncated step never updates the model on any rank, the step before the lagged host check
    raises ShardOverflowError."""
    v = words.to(torch.int64) & 0xFFFFFFFF  # the kernels' u32 counts
    nb = int(words.shape[1]) - 3 if nb is None else int(nb)
    counts, band_k, pc, cap = v[:, :nb], v[:, nb], v[:, nb + 1], v[:, nb + 2]
    bad = (counts > pc[:, None]).any(dim=1) | (band_k > cap)
    return bad.sum().to(torch.int32).reshape(1)


class _CountRing:
    """Each step's overflow words of EVERY rank -- per-band splat counts, band instance count and
    that rank's two capacities, (world, nb + 3) int32, gathered with the band images -- copied to
    pinned host memory without
    waiting, and checked a fixed number of steps later (``check_upto``), so that every rank checks
    the same steps at the same calls and raises for the same step."""

    def __init__(self, nb: int, device, ring: int = 4):
        self.pin = torch.cuda.is_available() and torch.device(device).type == "cuda"
        self.nb = nb
        self.ring = ring
        self.slots: list = []
        self.pending: list = []  # (step, slot, event or None, pair_cap, capacity)
        self.next = 0
        self.last = None  # (step, rows of words) of the latest checked step: its row statistics

    def push(self, step: int, words: torch.Tensor, pair_cap: int, capacity: int):
        """words: (world, nb + 3 [+ 3 grid_y]) int32 device tensor: every rank's counts, band K,
        pair_cap and capacity (each rank is checked against its own), then its row statistics."""
        if len(self.pending) == self.ring:
            self.check_upto(self.pending[0][0])  # the oldest, at the same step on every rank
        if len(self.slots) < self.ring or self.slots[self.next].shape != words.shape:
            slot = torch.zeros(words.shape, dtype=torch.int32, pin_memory=self.pin)
            if len(self.slots) < self.ring:
                self.slots.append(slot)
            else:
                self.slots[self.next] = slot
        slot = self.slots[self.next]
        self.next = (self.next + 1) % self.ring
        slot.copy_(words, non_blocking=True)
        ev = None
        if words.is_cuda:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(words.device))
        self.pending.append((step, slot, ev, pair_cap, capacity))

    def check_upto(self, last_step: int):
        """Wait for and check every entry up to step `last_step`; raise on an overflow."""
        while self.pending and self.pending[0][0] <= last_step:
            step, slot, ev, pair_cap, capacity = self.pending.pop(0)
            if ev is not None:
                ev.synchronize()
            nb = self.nb
            rows = [[int(x) & 0xFFFFFFFF for x in row] for row in slot.tolist()]  # u32
            for r, v in enumerate(rows):
                # rank r's words: its per-band counts, band K, then ITS pair_cap and capacity
                counts, band_k, pc, cap = v[:nb], v[nb], v[nb + 1], v[nb + 2]
                if max(counts) > pc or band_k > cap:
                    self.pending.clear()
                    raise ShardOverflowError(step, counts, pc, band_k, cap, rank=r)
            self.last = (step, rows)

    def poll(self):
        """Check every pending entry (waits for each)."""
        if self.pending:
            self.check_upto(self.pending[-1][0])


class ShardStep:
    """Forward + backward of one rank of the multi-GPU path (rasterizer.ShardRasterizer calls,
    the exchanges above in between).  `inputs`: the full Gaussian arrays (device tensors) --
    each rank reads only its shard's rows.  ``plan`` sizes the exchange once from a probe:
    the band cuts from the summed row histogram, ``pair_cap`` and the band's instance capacity
    from the true counts, each with ``headroom``.

    Overflow: a step whose splats exceed ``pair_cap`` (any send block's header count) or whose
    band holds more instances than ``capacity`` is truncated by the kernels.  Every rank's
    overflow words (its per-band splat counts and band instance count) ride in a footer row of
    the image all-gather, so every rank holds every rank's; they are copied to pinned memory
    without a host wait and checked ``lag`` steps later (or by ``check``), at the same call on
    every rank, so all ranks raise ``ShardOverflowError`` for the same step and none is left
    blocked in a collective (the C++ ``gsr::ShardStep`` does the same).  The same words also give
    ``overflow_guard`` after every step: a (1,) int32 device word, the number of ranks that
    overflowed in THAT step (``overflow_ranks``), identical on every rank and ready without a host
    wait.  A training loop passes ``(step.overflow_guard, 0)`` as the guard of its statistics and
    Adam step, so the truncated step's gradients are never applied on any rank, even before the
    lagged check raises.  ``live=True`` re-plans from the steps themselves: every step's shard
    row statistics (instances per tile row, rect start / end rows: GSR_FLAG_ROW_SPANS) ride in the
    same footer, and when step s - lag is checked every rank computes the cuts and capacities
    they call for (``plan_from_stats`` with headroom) and adopts them at that same call if the cuts
    moved, a capacity is short or one is over twice the need -- no probe, no collective, no wait
    beyond the lagged check (``live_replans`` counts them; the C++ step does the same).
    ``strict=True`` checks
    every step before returning it, at the cost of one host wait per step.  The caller
    re-plans (``plan``) and re-runs from that step.

    Moving cameras (training): ``set_camera`` renders from another view (same image size) from
    the next step on, and ``rebalance_every`` = M > 0 re-plans before every M-th step -- the
    row histogram, band cuts and capacities of the camera then in use (a collective every rank
    takes at the same step count, after the pending count checks under the old plan).  The
    reference's loop changes camera every iteration (train_utils.cpp:128-145), so a plan made
    once for the first camera drifts out of balance; M trades the probe's cost (two headers-only
    shard forwards, two all-reduces, one host wait) against that drift."""

    def __init__(self, rast, cam, inputs: dict, sh_degree: int, dist, group=None, headroom: float = 1.25,
                 strict: bool = False, rebalance_every: int = 0, lag: int = 2, live: bool = False):
        self.rast, self.cam, self.dist, self.group = rast, cam, dist, group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.D = sh_degree
        self.headroom = headroom
        self.strict = strict
        if rebalance_every < 0:
            raise ValueError("rebalance_every must be >= 0")
        self.rebalance_every = int(rebalance_every)
        if lag < 1:
            raise ValueError("lag must be >= 1")
        self.lag = int(lag)
        self.replans = 0
        self.live = bool(live)
        self.live_replans = 0
        self._stats_used = -1
        P = int(inputs["means3D"].shape[0])
        self.P = P
        self.g0, self.g1 = gaussian_shard(P, self.world, self.rank)
        self.shard = {k: (v[self.g0:self.g1] if v is not None else None) for k, v in inputs.items()}
        self.gy = (cam.height + TILE - 1) // TILE
        self.rows = equal_bands(self.gy, self.world)
        self.pair_cap = 0
        self.capacity = 0
        self.steps = 0
        self._ring = _CountRing(self.world, self.shard["means3D"].device)
        # buffers kept across steps (one stream: a step's kernels run after the previous step's)
        self._reuse = {"shard": {}, "band": {}, "grads": {}}

    def _shard_forward(self, pair_cap, row_hist=None):
        return self.rast.shard_forward(self.cam, self.rows, pair_cap, **self.shard, sh_degree=self.D,
                                       row_hist=row_hist, reuse=self._reuse["shard"] if pair_cap else None)

    def plan(self):
        """Probe (synchronous, setup only): balanced band cuts, then the pair capacity and the
        band's instance capacity.  The row histogram is u32 per shard on the device and summed
        over ranks in int64; a band above 2^31 - 1 instances is refused (int32 capacities)."""
        dev = self.shard["means3D"].device
        hist = torch.zeros(self.gy, dtype=torch.int32, device=dev)
        self._shard_forward(0, hist)  # pair_cap 0: headers only
        hist64 = hist.to(torch.int64) & 0xFFFFFFFF  # the kernel's u32 counts, widened before the sum
        self.dist.all_reduce(hist64, group=self.group)
        counts = hist64.cpu().numpy().astype(np.int64)
        self.rows = balance_bands(counts, self.world)
        sh = self._shard_forward(0)
        pc = sh.counts.to(torch.int64)
        self.dist.all_reduce(pc, op=self.dist.ReduceOp.MAX, group=self.group)
        self.pair_cap = round_up(max(int(pc.max()), 1) * self.headroom)
        band_k = [int(counts[self.rows[b]:self.rows[b + 1]].sum()) for b in range(self.world)]
        self.capacity = round_up(max(max(band_k), 1) * self.headroom)
        if self.capacity >= 2**31 or self.pair_cap * self.world >= 2**31:
            raise ValueError(f"band capacity {self.capacity} / pair_cap {self.pair_cap} exceed int32: use more ranks")
        self.band_instances = band_k
        self._ring.pending.clear()
        return self

    def set_camera(self, cam):
        """Render from `cam` from the next step on.  The band cuts and capacities stay those of the
        last plan until the next re-plan (``rebalance_every`` or an explicit ``plan()``); a step
        whose splats or band then exceed them raises ShardOverflowError as usual."""
        if (cam.width, cam.height) != (self.cam.width, self.cam.height):
            raise ValueError(f"camera size {cam.width}x{cam.height} != the plan's {self.cam.width}x{self.cam.height}")
        self.cam = cam

    @property
    def band(self) -> tuple[int, int]:
        return self.rows[self.rank], self.rows[self.rank + 1]

    def forward(self):
        # with live re-planning this shard's row statistics ride in the status footer (zeros
        # otherwise: the pack then skips its row-spans form)
        if getattr(self, "_stats", None) is None:
            self._stats = torch.zeros(3 * self.gy, dtype=torch.int32, device=self.shard["means3D"].device)
        if self.live:
            self._stats.zero_()
        sh = self.rast.shard_forward(self.cam, self.rows, self.pair_cap, **self.shard, sh_degree=self.D,
                                     row_hist=self._stats if self.live else None, row_spans=self.live,
                                     reuse=self._reuse["shard"])
        recv = all_to_all_blocks(sh.send, self.world, self.dist, self.group)
        st = self.rast.band_forward(self.cam, self.band, self.world, self.pair_cap, recv, self.capacity,
                                    reuse=self._reuse["band"])
        return sh, st

    def check(self):
        """Raise ShardOverflowError if any rank overflowed in a step so far.  Always waits for
        every pending step (a host sync); every rank must call it at the same step count."""
        self._ring.poll()

    def _replan_live(self):
        """Adopt the cuts / capacities the latest checked step's statistics call for (see the
        class doc); every rank takes the same decision from the same gathered words."""
        last = self._ring.last
        if last is None or last[0] == self._stats_used:
            return
        self._stats_used = last[0]
        nb, gy = self.world, self.gy
        o = nb + 3
        inst = np.zeros(gy, np.int64)
        starts, ends = [], []
        for v in last[1]:
            inst += np.asarray(v[o:o + gy], np.int64)
            starts.append(v[o + gy:o + 2 * gy])
            ends.append(v[o + 2 * gy:o + 3 * gy])
        rows, max_splats, band_k = plan_from_stats(inst, starts, ends, nb)
        pc_need, cap_need = max(max_splats, 1), max(max(band_k), 1)
        short = pc_need > self.pair_cap or cap_need > self.capacity
        fat = (self.pair_cap > 2 * round_up(pc_need * self.headroom)
               or self.capacity > 2 * round_up(cap_need * self.headroom))
        if rows == self.rows and not short and not fat:
            return
        pc, cap = round_up(pc_need * self.headroom), round_up(cap_need * self.headroom)
        if cap >= 2**31 or pc * self.world >= 2**31:
            raise ValueError(f"band capacity {cap} / pair_cap {pc} exceed int32: use more ranks")
        self.rows, self.pair_cap, self.capacity, self.band_instances = rows, pc, cap, band_k
        self.live_replans += 1

    def step(self, dL_dpix: torch.Tensor):
        """-> (full image, this shard's leaf gradients, shard state, band state).  Raises
        ShardOverflowError for an earlier step found to have overflowed (see the class doc).
        The returned gradients and states live in buffers the next step reuses: consume them
        (e.g. the optimizer step) before calling step() again."""
        if self.rebalance_every and self.steps and self.steps % self.rebalance_every == 0:
            self._ring.poll()  # the old plan's pending checks first
            self.plan()
            self.replans += 1
        # the step `lag` steps back, on every rank at this same call (its words have long landed)
        self._ring.check_upto(self.steps - self.lag)
        if self.live:
            self._replan_live()
        sh, st = self.forward()
        # this rank's overflow words ride in the image all-gather: every rank checks every rank's
        key = (self.pair_cap, self.capacity)
        if getattr(self, "_caps_key", None) != key:  # a device copy of the capacities, made once per plan
            self._caps = torch.tensor(list(key), dtype=torch.int32, device=sh.counts.device)
            self._caps_key = key
        words = torch.cat([sh.counts.reshape(-1), st.k_device().reshape(-1), self._caps, self._stats]).to(torch.int32)
        img = ImageGather(st.color, self.rows, self.rank, self.dist, self.group, status=words)  # overlaps B1
        g2 = self.rast.band_backward(st, self.world, self.pair_cap, dL_dpix, reuse=self._reuse["band"])
        back = all_to_all_blocks(g2, self.world, self.dist, self.group)
        grads = self.rast.shard_backward(sh, back, reuse=self._reuse["grads"])
        out = img.wait(), grads, sh, st
        allw = img.statuses()
        # the step's agreement word on the device (same value on every rank): the optimizer guard
        if getattr(self, "overflow_guard", None) is None or self.overflow_guard.device != allw.device:
            self.overflow_guard = torch.zeros(1, dtype=torch.int32, device=allw.device)
        self.overflow_guard.copy_(overflow_ranks(allw, self.world))
        self._ring.push(self.steps, allw, self.pair_cap, self.capacity)
        self.steps += 1
        if self.strict:
            self._ring.poll()
        return out


def simulate_ranks(rast, cam, inputs: dict, sh_degree: int, world: int, dL_dpix: torch.Tensor,
                   headroom: float = 1.25, rows=None, timer=None, pair_cap=None, capacity=None):
    """Every rank's compute of one multi-GPU step, in one process on one GPU, with the
    collectives replaced by block copies (same layouts as the RCCL exchange): the rehearsal of
    scripts/band_sim.py and the GPU parity tests.  `timer(name, rank, fn)` (optional) wraps each
    per-rank call.  `pair_cap` / `capacity` override the probed capacities (overflow tests).
    Returns (image, leaf gradients of all P, plan dict); the plan's ``overflow`` lists the
    (rank, per-band counts, band K) of every rank whose step exceeded them."""
    run = timer or (lambda name, r, fn: fn())
    P = int(inputs["means3D"].shape[0])
    gy = (cam.height + TILE - 1) // TILE
    shards = [gaussian_shard(P, world, r) for r in range(world)]
    sub = lambda r: {k: (v[shards[r][0]:shards[r][1]] if v is not None else None) for k, v in inputs.items()}
    dev = inputs["means3D"].device
    if rows is None:  # probe 1: row histogram over all shards -> balanced cuts
        hist = torch.zeros(gy, dtype=torch.int32, device=dev)
        for r in range(world):
            rast.shard_forward(cam, equal_bands(gy, world), 0, **sub(r), sh_degree=sh_degree, row_hist=hist)
        counts = hist.cpu().numpy().astype(np.int64)
        rows = balance_bands(counts, world)
    else:
        hist = torch.zeros(gy, dtype=torch.int32, device=dev)
        for r in range(world):
            rast.shard_forward(cam, rows, 0, **sub(r), sh_degree=sh_degree, row_hist=hist)
        counts = hist.cpu().numpy().astype(np.int64)
    if pair_cap is None:
        pc = max(int(rast.shard_forward(cam, rows, 0, **sub(r), sh_degree=sh_degree).counts.max())
                 for r in range(world))
        pair_cap = round_up(max(pc, 1) * headroom)
    if capacity is None:
        capacity = round_up(max(max(int(counts[rows[b]:rows[b + 1]].sum()) for b in range(world)), 1) * headroom)
    shs = [run("shard_forward", r, lambda r=r: rast.shard_forward(cam, rows, pair_cap, **sub(r), sh_degree=sh_degree))
           for r in range(world)]
    blk = shs[0].send.numel() // world
    image = torch.zeros((3, cam.height, cam.width), dtype=torch.float32, device=dev)
    back_parts = [[None] * world for _ in range(world)]  # [src][band]
    bsts = []
    for b in range(world):
        recv = torch.cat([shs[r].send[b * blk:(b + 1) * blk] for r in range(world)])
        st = run("band_forward", b, lambda b=b, recv=recv: rast.band_forward(cam, (rows[b], rows[b + 1]), world,
                                                                                pair_cap, recv, capacity,
                                                                                out_color=image))
        g2 = run("band_backward", b, lambda st=st: rast.band_backward(st, world, pair_cap, dL_dpix))
        for r in range(world):
            back_parts[r][b] = g2[r * pair_cap:(r + 1) * pair_cap]
        bsts.append(st)
    # the gradient all-to-all: rank r receives band b's rows for its splats (a contiguous receive
    # buffer, as the collective writes it -- the copy is the exchange, outside the compute timer)
    grad_recv = [torch.cat(back_parts[r]) for r in range(world)]
    grads = [run("shard_backward", r, lambda r=r: rast.shard_backward(shs[r], grad_recv[r])) for r in range(world)]
    full = {k: torch.cat([g[k] for g in grads]) for k in grads[0]}
    overflow = []
    for r in range(world):
        cnt = [int(c) for c in shs[r].counts.tolist()]
        k = int(bsts[r].k_device().item())
        if max(cnt) > pair_cap or k > capacity:
            overflow.append((r, cnt, k))
    return image, full, dict(rows=rows, pair_cap=pair_cap, capacity=capacity, shards=shs, bands=bsts,
                             band_instances=[int(counts[rows[b]:rows[b + 1]].sum()) for b in range(world)],
                             overflow=overflow)
