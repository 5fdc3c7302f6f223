"""Multi-GPU image tiling and reassembly after the gather.  SURVEY.md 8(e): pixels are
independent, the voxel store is replicated per GPU, and the only exchange is the final
gather of the framebuffer to rank 0.  Two layouts (include/vr.h):

  row bands -- band b of band_rows rows -> rank b % R (vr_render_bands);
  2-D tiles -- every band cut into column blocks of tile_cols pixels, block j of band b ->
               rank (j + stride * b) % R (vr_render_tiles): every rank gets a share of every
               band, so a cluster of expensive rows (C5's crawl rows) is spread over all ranks
               while each 8x8 wave tile stays whole.
"""
from __future__ import annotations

import contextlib
import math

import torch

from .renderer import band_buffer_words


def bands_per_rank(height: int, band_rows: int, nranks: int) -> int:
    nb = -(-height // band_rows)
    return -(-nb // nranks)


def assemble_bands(parts: torch.Tensor, width: int, height: int, band_rows: int) -> torch.Tensor:
    """parts: [R, words] per-rank band buffers (vr_render_bands layout) -> [height, width] frame."""
    R = parts.shape[0]
    per = bands_per_rank(height, band_rows, R)
    expect = band_buffer_words(width, height, band_rows, R)
    if parts.shape[1] != expect or per * band_rows * width != expect:
        raise ValueError(f"band buffers have {parts.shape[1]} words, expected {expect}")
    img = parts.reshape(R, per, band_rows, width).permute(1, 0, 2, 3).reshape(per * R * band_rows, width)
    return img[:height]


def deal_stride(nranks: int, stride: int = 0) -> int:
    """The 2-D deal's stride as the library uses it (vr_deal_stride_default for 0)."""
    s = stride or (1 if nranks % 3 == 0 else 3)
    return s % nranks


def tile_local_width(width: int, tile_cols: int, nranks: int) -> int:
    """Words per local row of a 2-D tile buffer: this rank's column blocks of one band."""
    nblk = -(-width // tile_cols)
    return -(-nblk // nranks) * tile_cols


def tile_words(width: int, height: int, band_rows: int, tile_cols: int, nranks: int) -> int:
    """vr_tile_buffer_words (the same arithmetic, without the library)."""
    return -(-height // band_rows) * band_rows * tile_local_width(width, tile_cols, nranks)


def tile_source_index(width: int, height: int, band_rows: int, tile_cols: int, nranks: int,
                      stride: int = 0) -> torch.Tensor:
    """For every frame pixel (row-major), its index in the nranks tile buffers laid back to back:
    the inverse of the 2-D deal (vr_internal.h KView, vr_march.hip assemble_tiles_kernel)."""
    s = deal_stride(nranks, stride)
    words = tile_words(width, height, band_rows, tile_cols, nranks)
    lw = tile_local_width(width, tile_cols, nranks)
    y = torch.arange(height, dtype=torch.int64)[:, None]
    x = torch.arange(width, dtype=torch.int64)[None, :]
    b, j = y // band_rows, x // tile_cols
    rank = (j + s * (b % nranks)) % nranks
    lx = (j // nranks) * tile_cols + x % tile_cols
    return (rank * words + y * lw + lx).reshape(-1)


def assemble_tiles(parts: torch.Tensor, width: int, height: int, band_rows: int, tile_cols: int,
                   stride: int = 0) -> torch.Tensor:
    """parts: [R, words * px] per-rank tile buffers (px elements per pixel) -> [height, width * px].
    (Host-side form for CPU tests; rank 0 on a GPU uses vr_assemble_tiles.)"""
    R = parts.shape[0]
    words = tile_words(width, height, band_rows, tile_cols, R)
    px, rem = divmod(parts.shape[1], words)
    if rem or px < 1:
        raise ValueError(f"tile buffers have {parts.shape[1]} elements, expected a multiple of {words}")
    idx = tile_source_index(width, height, band_rows, tile_cols, R, stride).to(parts.device)
    return parts.reshape(R * words, px).index_select(0, idx).reshape(height, width * px)


def tile_rank_buffer(frame: torch.Tensor, rank: int, nranks: int, band_rows: int, tile_cols: int,
                     stride: int = 0) -> torch.Tensor:
    """What rank `rank` renders of `frame` [H, W] in the 2-D deal (0 past the frame): for tests."""
    H, W = frame.shape
    words = tile_words(W, H, band_rows, tile_cols, nranks)
    idx = tile_source_index(W, H, band_rows, tile_cols, nranks, stride)
    mine = (idx // words) == rank
    buf = torch.zeros(words, dtype=frame.dtype)
    buf[idx[mine] - rank * words] = frame.reshape(-1)[mine]
    return buf


def strip_bounds(row_cost, nranks: int, align: int = 8) -> list[int]:
    """The cost-balanced contiguous deal (round 6): cut rows [0, H) into nranks strips of
    about equal cost -- rank r renders rows [b[r], b[r+1]) -- from a cost per row (any
    non-negative weights, len = H).  Every boundary but H is a multiple of `align` rows and
    every strip holds at least one aligned block.  A strip is the most compact share of the
    frame a rank can have (its waves walk neighbouring rays: a rank of 8 issues its pixels
    ~13 % more efficiently than with the 2-D tile deal, profiles/r06/deal/), and equal costs
    keep the ranks balanced, which equal-height strips are not (C5: 0.040-0.117 ms)."""
    H = len(row_cost)
    nblk = -(-H // align)
    if nranks < 1 or nblk < nranks:
        raise ValueError(f"{H} rows in blocks of {align} cannot be cut into {nranks} strips")
    blk = [float(sum(row_cost[i * align:(i + 1) * align])) for i in range(nblk)]
    cum = [0.0]
    for c in blk:
        cum.append(cum[-1] + max(c, 0.0))
    # the contiguous partition that minimises the costliest strip (exact dynamic programme over
    # block edges: best[k][e] = the least possible max cost of k strips covering blocks [0, e))
    inf = float("inf")
    best = [[inf] * (nblk + 1) for _ in range(nranks + 1)]
    arg = [[0] * (nblk + 1) for _ in range(nranks + 1)]
    best[0][0] = 0.0
    for k in range(1, nranks + 1):
        prev, cur, ak = best[k - 1], best[k], arg[k]
        for e in range(k, nblk - (nranks - k) + 1):
            m, mj = inf, k - 1
            for j in range(e - 1, k - 2, -1):       # the last strip is blocks [j, e)
                last = cum[e] - cum[j]
                if last >= m:
                    break                           # (only grows as j falls)
                v = prev[j] if prev[j] > last else last
                if v < m:
                    m, mj = v, j
            cur[e], ak[e] = m, mj
    cuts, e = [nblk], nblk
    for k in range(nranks, 0, -1):
        e = arg[k][e]
        cuts.append(e)
    cuts.reverse()
    return [c * align for c in cuts[:-1]] + [H]


def rebalance_strips(bounds, times, align: int = 8, prior=None, damping: float = 0.5):
    """One step of the learned strip deal: from the strips `bounds` and each rank's measured
    time for its strip, a cost per row (time / height, uniform within each strip), averaged
    with the previous estimate `prior` (a per-row cost list, weight `damping` on the new
    one) and re-cut by strip_bounds.  Returns (new bounds, the per-row cost estimate)."""
    H = bounds[-1]
    est = [0.0] * H
    for r in range(len(bounds) - 1):
        h = bounds[r + 1] - bounds[r]
        for y in range(bounds[r], bounds[r + 1]):
            est[y] = float(times[r]) / h
    if prior is not None:
        est = [damping * e + (1.0 - damping) * p for e, p in zip(est, prior)]
    return strip_bounds(est, len(bounds) - 1, align), est


def assemble_strips(parts: torch.Tensor, bounds, width: int, px: int = 1) -> torch.Tensor:
    """parts: [R, >= max_h * width * px] per-rank strip buffers (rank r's rows [b[r], b[r+1])
    first, padding after) -> [H, width * px] frame.  (Rank 0 on a GPU does the same copies.)"""
    H = bounds[-1]
    out = torch.empty((H, width * px), dtype=parts.dtype, device=parts.device)
    for r in range(len(bounds) - 1):
        h = bounds[r + 1] - bounds[r]
        out[bounds[r]:bounds[r + 1]] = parts[r, :h * width * px].view(h, width * px)
    return out


def owned_rows(height: int, band_rows: int, rank: int, nranks: int) -> list[int]:
    """Frame rows rendered by `rank` (for tests and accounting)."""
    rows = []
    nb = -(-height // band_rows)
    for b in range(rank, nb, nranks):
        rows.extend(range(b * band_rows, min(height, (b + 1) * band_rows)))
    return rows


def frame_resolution(width: int, height: int, nranks: int, tiling: str) -> tuple[int, int]:
    """The frame N ranks render together: "fixed" -- the config's own frame cut into
    bands over the ranks (BASELINE C5: one 3840x2160 frame tiled over 8 GPUs; strong
    scaling); "weak" -- the same view at about N x the pixels (weak_scaled_resolution)."""
    if tiling == "fixed":
        return width, height
    if tiling == "weak":
        return weak_scaled_resolution(width, height, nranks)
    raise ValueError(f"unknown tiling {tiling!r}")


def pipeline_depth(config: str) -> int:
    """Frames in flight for a BASELINE config (BandGather's depth).  C5's frames end in
    a crawl pass -- a latency chain of ~0.3-0.5 ms whatever the rank's share of the
    frame -- so its pipeline must hold enough frames to cover that chain: 8 (one GPU:
    0.670 vs 0.710 ms per frame at 3; one rank of 8, fixed tiling: 0.125 vs 0.205 ms,
    profiles/r03/queues/, profiles/r03/proj/).  The other configs' frames end in a few
    long tile-pass waves that one more frame covers: 2 (3 and 4 measured slower)."""
    return 8 if config == "C5" else 2


def pipeline_hw_queues(depth: int, nranks: int = 1) -> int:
    """Hardware queues a process needs so that its busy streams never share one: two
    streams on one queue run one after the other (the box's default is 4 queues per
    process; measured: C5 at 4 frames in flight on 4 queues ran slower than at 3).  The
    streams: one per frame in flight, the null stream, and with N > 1 ranks rank 0's
    assembly stream and the RCCL communicator's stream.  0 = the default suffices."""
    streams = depth + 1 + (2 if nranks > 1 else 0)
    return 16 if streams > 4 else 0


def init_frame_group(world: int, local_rank: int, backend: str = "auto", same_device: bool = False,
                     force_group: bool = False):
    """The device and process group of one rank of the frame pipeline (bench.py's N > 1
    path).  backend "auto"/"nccl": RCCL over xGMI, one GPU per rank (RCCL refuses two ranks
    on one device).  "gloo": the same pipeline with the gather staged through host memory
    (BandGather(stage_host=True)) -- what lets N ranks share one GPU (same_device: every
    rank on cuda:0) to run the multi-rank path on a one-GPU box.
    Returns (device, backend, stage_host); world == 1 starts no group unless force_group
    (bench.py --exchange: one rank through the whole N > 1 path, RCCL included)."""
    import torch.distributed as dist
    dev_index = 0 if same_device else local_rank
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    if backend == "auto":
        backend = "nccl"
    if backend not in ("nccl", "gloo"):
        raise ValueError(f"unknown backend {backend!r}")
    if same_device and world > 1 and backend == "nccl":
        raise ValueError("several ranks on one GPU need the gloo backend (RCCL refuses a duplicate GPU)")
    if world > 1 or force_group:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    return dev, backend, backend == "gloo"


def weak_scaled_resolution(width: int, height: int, nranks: int) -> tuple[int, int]:
    """The same view at about nranks x the pixels (both sides x sqrt(nranks), so the
    aspect ratio -- and with it Camera::Camera's view -- stays put and every rank
    renders about width x height pixels).  nranks = 1 gives (width, height)."""
    f = math.sqrt(nranks)
    return int(round(width * f)), int(round(height * f))


class BandGather:
    """Image tiling across ranks (row bands, or the 2-D tile deal with tile_cols > 0), with
    frames in flight.

    step(render) renders this rank's bands of the next frame into one of `depth`
    band buffers and starts an asynchronous gather of it to rank 0 (RCCL on
    GPUs, gloo on CPU); rank 0 then assembles the frame into `frame` (one
    permuting copy).  On GPUs every buffer slot has its own stream: the render of
    frame k+1 does not wait for frame k (the few long waves that end a frame
    overlap the start of the next one), frame k's gather runs beside frame k+1's
    render, and rank 0's assembly copies run on a side stream beside both.  A
    slot is reused `depth` frames later, after its gather (and, on rank 0, its
    copy) has completed.  drain() completes every outstanding frame and joins
    all streams into the caller's.  With one rank the band buffer already is
    the frame (bands in row order) and nothing is exchanged.
    """

    def __init__(self, width: int, height: int, band_rows: int, rank: int, nranks: int,
                 device, depth: int = 2, on_frame=None, rgb8: bool = False, stage_host: bool = False,
                 tile_cols: int = 0, stride: int = 0, exchange: bool | None = None, strips=None):
        self.W, self.H, self.B = width, height, band_rows
        self.rank, self.R, self.depth = rank, nranks, depth
        # exchange: gather every frame to rank 0 and assemble it there (N > 1; with one rank it
        # is forced only to run that code -- RCCL included -- on a one-GPU box)
        self.x = nranks > 1 if exchange is None else bool(exchange)
        x = self.x
        # strips (round 6, the learned cost-balanced contiguous deal): rank r renders rows
        # [strips[r], strips[r+1]) into the first rows of its buffer; every buffer holds the
        # tallest strip (one gather of equal buffers) and rank 0 copies each strip into place
        self.S = list(strips) if (strips is not None and x) else None
        if self.S is not None and (len(self.S) != nranks + 1 or self.S[0] != 0 or self.S[-1] != height or
                                   any(self.S[i] >= self.S[i + 1] for i in range(nranks))):
            raise ValueError(f"strips {strips} do not cut rows [0, {height}) into {nranks} strips")
        # the 2-D tile deal (with the exchange only: without it the band buffer is the frame)
        self.T = int(tile_cols) if (x and self.S is None) else 0
        self.stride = deal_stride(nranks, stride) if self.T else 0
        words = (width * max(self.S[i + 1] - self.S[i] for i in range(nranks)) if self.S is not None else
                 tile_words(width, height, band_rows, self.T, nranks) if self.T else
                 band_buffer_words(width, height, band_rows, nranks))
        self.device = device
        self.xdt = torch.uint8 if (bool(rgb8) and x) else torch.int32
        # stage_host (a gloo group over GPU buffers -- gloo gathers host tensors only, e.g.
        # several ranks sharing one GPU, where RCCL refuses): each frame's send buffer is
        # copied to pinned host memory once its render is complete, gathered there, and the
        # receive buffers are copied back to the device before the same assembly
        self.stage = bool(stage_host) and x and torch.device(device).type == "cuda"
        # rgb8 (GPUs, N > 1): the bands travel as the RGB8 framebuffer (3 B per pixel
        # instead of the 4-B packed word: a quarter less over xGMI) and rank 0
        # assembles an RGB8 frame [H, W, 3]
        self.rgb8 = bool(rgb8) and x
        self.px = 3 if self.rgb8 else 1                  # elements per pixel in the exchanged buffers
        self.per = bands_per_rank(height, band_rows, nranks)
        self._alloc(words)
        frame_rows = height if (self.T or self.S is not None) else self.per * nranks * band_rows
        self.frame = (torch.empty((frame_rows, width * self.px), dtype=self.xdt, device=device)
                      if rank == 0 else None)
        self.work = [None] * depth
        dev = torch.device(device)
        cuda = dev.type == "cuda"
        self.streams = [torch.cuda.Stream(dev) for _ in range(depth)] if cuda else None
        # rank 0: the un-interleaving copy on a side stream (the render is latency-bound,
        # the copy HBM-bound); a receive buffer is gathered into again only after its
        # copy has finished.
        self.side = torch.cuda.Stream(dev) if (cuda and rank == 0 and x) else None
        self.copied = [None] * depth
        self.joins = [None] * depth  # per slot: the event its stream waits on for the caller's work
        self.pending = []            # slots in submission order
        self.on_frame = on_frame     # rank 0: callback(frame[:H]) after each assembled frame
        self.k = 0
        self.last = 0                # the slot of the latest step

    def _alloc(self, words: int) -> None:
        """The per-slot buffers of `words` pixels per rank (band buffers, RGB8 send buffers, rank
        0's receive buffers, pinned staging buffers)."""
        depth, nranks, device, xdt = self.depth, self.R, self.device, self.xdt
        self.words = words
        self.bufs = [torch.empty(words, dtype=torch.int32, device=device) for _ in range(depth)]
        self.packed = ([torch.empty(words * 3, dtype=torch.uint8, device=device) for _ in range(depth)]
                       if self.rgb8 else None)
        self.recv = ([torch.empty((nranks, words * self.px), dtype=xdt, device=device) for _ in range(depth)]
                     if (self.rank == 0 and self.x) else None)
        if self.stage:
            self.h_send = [torch.empty(words * self.px, dtype=xdt, pin_memory=True) for _ in range(depth)]
            self.h_recv = ([torch.empty((nranks, words * self.px), dtype=xdt, pin_memory=True) for _ in range(depth)]
                           if self.rank == 0 else None)

    def set_strips(self, strips) -> None:
        """Re-cut the strip deal (learned strips: bench.py re-cuts them from the ranks' measured
        frame times before timing); only between drained frames.  Buffers are re-made for the
        new tallest strip; the streams are kept."""
        if self.S is None:
            raise ValueError("not a strip deal")
        if self.pending:
            raise RuntimeError("set_strips with frames in flight: drain() first")
        S = list(strips)
        if len(S) != self.R + 1 or S[0] != 0 or S[-1] != self.H or any(S[i] >= S[i + 1] for i in range(self.R)):
            raise ValueError(f"strips {strips} do not cut rows [0, {self.H}) into {self.R} strips")
        if self.streams is not None:
            torch.cuda.synchronize(self.device)        # (the old buffers' last users are done)
        self.S = S
        self._alloc(self.W * max(S[i + 1] - S[i] for i in range(self.R)))

    def rows(self) -> tuple[int, int]:
        """This rank's strip (strip deal only)."""
        return self.S[self.rank], self.S[self.rank + 1]

    def _slot_stream(self, slot: int):
        return torch.cuda.stream(self.streams[slot]) if self.streams is not None else contextlib.nullcontext()

    def _assemble(self, slot: int) -> None:
        rw = self.W * self.px
        if self.S is not None:                             # one copy per strip
            for r in range(self.R):
                y0, y1 = self.S[r], self.S[r + 1]
                self.frame[y0:y1].copy_(self.recv[slot][r, :(y1 - y0) * rw].view(y1 - y0, rw))
        elif self.T:
            if self.recv[slot].is_cuda:                    # one un-dealing kernel (vr_assemble_tiles)
                from .renderer import assemble_tiles_device
                eb = self.px * self.recv[slot].element_size()
                assemble_tiles_device(self.recv[slot], self.frame, eb, self.W, self.H, self.B, self.T, self.R,
                                      self.stride)
            else:
                self.frame.copy_(assemble_tiles(self.recv[slot], self.W, self.H, self.B, self.T, self.stride))
        else:
            src = self.recv[slot].view(self.R, self.per, self.B, rw).permute(1, 0, 2, 3)
            self.frame.view(self.per, self.R, self.B, rw).copy_(src)
        if self.on_frame is not None:
            f = self.frame[:self.H]
            self.on_frame(f.view(self.H, self.W, 3) if self.rgb8 else f)

    def _finish(self, slot: int) -> None:
        if not self.x and self.on_frame is None:     # nothing to hand over (the bench's loop)
            self.pending.remove(slot)
            return
        with self._slot_stream(slot):
            if not self.x:
                if self.on_frame is not None:
                    self.on_frame(self.bufs[slot].view(-1, self.W)[:self.H])
            else:
                self.work[slot].wait()      # the slot's stream: bufs[slot] may be rendered into again
                self.work[slot] = None
                if self.stage and self.rank == 0:
                    self.recv[slot].copy_(self.h_recv[slot], non_blocking=True)
                if self.rank == 0:
                    if self.side is not None:
                        self.side.wait_stream(self.streams[slot])
                        with torch.cuda.stream(self.side):
                            self._assemble(slot)
                            ev = torch.cuda.Event()
                            ev.record(self.side)
                        self.copied[slot] = ev
                    else:
                        self._assemble(slot)
        self.pending.remove(slot)

    def step(self, render) -> None:
        """render(buf) enqueues this rank's bands on the current stream (or, with a
        `vr_stream_arg` attribute and no exchange, render(buf, stream) on the given one)."""
        slot = self.k % self.depth
        if slot in self.pending:
            self._finish(slot)
        if self.streams is not None and self.k < self.depth:
            # the slot's stream picks up after the caller's work (inputs, earlier frames' users);
            # one made event per slot, recorded again each time (wait_stream makes a new one)
            if self.joins[slot] is None:
                self.joins[slot] = torch.cuda.Event()
            self.joins[slot].record(torch.cuda.current_stream())
            self.streams[slot].wait_event(self.joins[slot])
        if not self.x and self.streams is not None and getattr(render, "vr_stream_arg", False):
            # a render that takes the stream (renderer.PreparedRender): no torch stream context,
            # the host path of a frame is one ctypes call
            render(self.bufs[slot], self.streams[slot])
            self.pending.append(slot)
            self.last = slot
            self.k += 1
            return
        with self._slot_stream(slot):
            render(self.bufs[slot])
            if self.x:
                import torch.distributed as dist
                send = self.bufs[slot]
                if self.rgb8:
                    from .renderer import pack_rgb8
                    send = pack_rgb8(self.bufs[slot], out=self.packed[slot])
                dst = list(self.recv[slot].unbind(0)) if self.rank == 0 else None
                if self.copied[slot] is not None:       # its previous frame has left recv[slot]
                    torch.cuda.current_stream().wait_event(self.copied[slot])
                    self.copied[slot] = None
                if self.stage:
                    # (the host buffers are free: this slot's previous gather was waited on,
                    # and on rank 0 its copy-back is ordered before this frame's copy-out)
                    self.h_send[slot].copy_(send, non_blocking=True)
                    torch.cuda.current_stream().synchronize()
                    send = self.h_send[slot]
                    dst = list(self.h_recv[slot].unbind(0)) if self.rank == 0 else None
                self.work[slot] = dist.gather(send, dst, dst=0, async_op=True)
        self.pending.append(slot)
        self.last = slot
        self.k += 1

    def last_frame(self) -> torch.Tensor:
        """After drain(): rank 0's last frame -- [H, W, 3] uint8 RGB8 when the bands travel
        as RGB8, else [H, W] packed words (the band buffer itself with one rank)."""
        if not self.x:
            return self.bufs[self.last].view(-1, self.W)[:self.H]
        f = self.frame[:self.H]
        return f.view(self.H, self.W, 3) if self.rgb8 else f

    def drain(self) -> None:
        while self.pending:
            self._finish(self.pending[0])
        if self.streams is not None:                 # the caller's stream sees every frame complete
            cur = torch.cuda.current_stream()
            for st in self.streams:
                cur.wait_stream(st)
            if self.side is not None:
                cur.wait_stream(self.side)
        self.k = 0
