"""Streaming multi-view reconstruction: host ingest, H2D, decode + triangulate
and D2H of the clouds overlapped, for scans whose stacks live on the host.

The reference processes one scan folder at a time, end to end and serially
(multi_point_cloud_process.py:201-257 for a turntable batch;
server/sl_system.py:483-694 per view).  On MI355X the kernels take ~0.1 ms
per 4K view while one 4K stack is 381 MB of host data, so the rate of a
host-resident scan is set by PCIe and by host-side image decoding, not by the
kernels.  ``ViewPipeline`` keeps all three engines busy at once:

  host thread     fill(i) decodes / copies view i into a pinned slot
  copy stream     H2D of slot k                     (hipMemcpyAsync, pinned)
  compute stream  k_decode / k_count / k_cloud on slot k (after its H2D event)
  D2H thread      waits for slot k's compute event, copies its points back
                  into pinned memory, hands them to consume(i, xyz, bgr) in
                  view order, then frees slot k

with ``slots`` (default 3) stacks in flight.  Only the planes the cloud reads
are uploaded: white, black and the column (pattern, inverse) pairs --
reconstruct_point_cloud never reads row_map (sl_system.py:584-653), so the
2 * n_rows_bits row planes are neither decoded from disk nor sent over PCIe
(24 of 46 planes for 11 + 11 bits).  The full file count is still validated
with gray_decode's rules (sl_system.py:515-516, 549-554): ValueError below
4 files, IndexError for a pattern without its inverse.  The arithmetic is the
same library call as ``Reconstructor.decode_triangulate``, so the clouds are
bit-identical to the one-shot path.
"""
from __future__ import annotations

import queue
import threading
import time
from dataclasses import dataclass, field

import numpy as np
import torch

from . import core


def bit_count(n: int) -> int:
    """ceil(log2(n)) as gray_decode computes it (sl_system.py:545)."""
    return int(np.ceil(np.log2(n))) if n > 1 else 0


def planes_for_cloud(n_img: int, n_cols: int = 1920, n_rows: int = 1080) -> int:
    """Number of leading stack files the cloud needs, after checking the whole
    stack of ``n_img`` files with gray_decode's rules (the library's own
    checks on the full stack, sl_decode_triangulate)."""
    if n_img < 4:
        raise ValueError("Not enough images in folder to decode.")
    nc, nr = bit_count(n_cols), bit_count(n_rows)
    idx = 2
    for _ in range(nc + nr):
        if idx >= n_img:
            break
        if idx + 1 >= n_img:
            raise IndexError("list index out of range")
        idx += 2
    return min(n_img, 2 + 2 * nc)


@dataclass
class PipelineStats:
    views: int = 0
    pixels: int = 0
    points: int = 0
    h2d_bytes: int = 0
    d2h_bytes: int = 0
    wall_s: float = 0.0
    fill_s: float = 0.0        # host time inside fill()
    consume_s: float = 0.0     # D2H-thread time inside consume()
    per_view_points: list = field(default_factory=list)

    def as_dict(self) -> dict:
        w = max(self.wall_s, 1e-12)
        return {"views": self.views, "pixels": self.pixels, "points": self.points, "wall_s": self.wall_s,
                "px_per_s": self.pixels / w, "h2d_GBps": self.h2d_bytes / w / 1e9,
                "d2h_GBps": self.d2h_bytes / w / 1e9, "fill_s": self.fill_s, "consume_s": self.consume_s}


@dataclass
class HostView:
    """A view already in pinned host memory: ``stack`` uint8 [>= n_up, H, W]
    (only its first n_up planes are read), ``texture`` uint8 [H, W, 3] BGR or
    None (the white plane replicated)."""
    stack: torch.Tensor
    texture: torch.Tensor | None = None


class ViewPipeline:
    """Overlapped host -> device -> host processing of equally sized views.

    ``fill(i, stack, texture) -> bool`` writes view i into the pinned uint8
    tensors ``stack`` [n_up, H, W] (the first n_up files of the view, n_up =
    ``planes_for_cloud``) and ``texture`` [H, W, 3] BGR, and returns True when
    the texture is the white plane replicated (single-channel file 0, what
    cv2.imread gives), in which case no texture is uploaded.  ``fill`` may
    instead return a ``HostView`` of caller-owned pinned tensors (e.g. frames
    a capture driver already placed in pinned memory): they are uploaded as
    they are, and must stay unchanged until ``consume`` has seen view i.
    ``consume(i, xyz, bgr)`` receives view i's points (numpy views of pinned
    memory, valid during the call) in view order, on the D2H thread.

    Device-resident consumers: ``on_device(i, xyz, bgr)`` receives view i's
    points as device tensors (slices of the slot's output, valid during the
    call; the D2H stream is current, so copies the callback enqueues are
    ordered before the slot is reused).  With ``consume=None`` the points never
    leave HBM -- only the 16-byte view offsets come back, to size the slices.
    ``poses`` (device or host [n_views, 4, 4] f64): view i is moved by
    ``poses[i]`` inside k_cloud (the f64 pose epilogue of decode_triangulate).
    ``count_masked``: the kernels also count each view's masked-in pixels (the
    N of "Processing N valid pixels...", sl_system.py:601-602);
    ``masked_count(i)`` returns view i's inside ``consume`` / ``on_device``.
    """

    def __init__(self, engine: core.Reconstructor, *, H: int, W: int, n_img: int, n_cols: int = 1920,
                 n_rows: int = 1080, mask_mode: str = "adaptive", xyz_dtype=torch.float64,
                 fast_f32: bool = False, slots: int = 3, count_masked: bool = False):
        if slots < 2:
            raise ValueError("slots must be >= 2")
        self.eng = engine
        self.H, self.W = int(H), int(W)
        self.n_cols, self.n_rows = int(n_cols), int(n_rows)
        self.n_img = int(n_img)
        self.n_up = planes_for_cloud(self.n_img, self.n_cols, self.n_rows)
        self.mask_mode = mask_mode
        self.xyz_dtype = xyz_dtype
        self.fast_f32 = fast_f32
        self.slots = slots
        dev = engine.device
        px = self.H * self.W
        self._copy = torch.cuda.Stream(dev)
        self._compute = torch.cuda.Stream(dev)
        self._d2h = torch.cuda.Stream(dev)
        esz = torch.empty((), dtype=xyz_dtype).element_size()
        self._hs = [torch.empty((self.n_up, self.H, self.W), dtype=torch.uint8, pin_memory=True) for _ in range(slots)]
        self._ht = [torch.empty((self.H, self.W, 3), dtype=torch.uint8, pin_memory=True) for _ in range(slots)]
        self._ds = [torch.empty((self.n_up, self.H, self.W), dtype=torch.uint8, device=dev) for _ in range(slots)]
        self._dt = [torch.empty((self.H, self.W, 3), dtype=torch.uint8, device=dev) for _ in range(slots)]
        self._hx = [torch.empty((px, 3), dtype=xyz_dtype, pin_memory=True) for _ in range(slots)]
        self._hb = [torch.empty((px, 3), dtype=torch.uint8, pin_memory=True) for _ in range(slots)]
        self._hn = [torch.empty(3, dtype=torch.int64, pin_memory=True) for _ in range(slots)]
        self.count_masked = bool(count_masked)
        self._mc = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(slots)]
        self._masked: dict = {}
        self._out = [{} for _ in range(slots)]
        self._esz = esz
        engine.reserve(1, px)

    def masked_count(self, i: int) -> int:
        """View i's masked-in pixel count (``count_masked``), valid from its
        ``consume`` / ``on_device`` call until ``run`` returns."""
        return self._masked[i]

    def run(self, n_views: int, fill, consume=None, *, on_device=None, poses=None) -> PipelineStats:
        st = PipelineStats()
        if poses is not None:
            poses = torch.as_tensor(poses, dtype=torch.float64).reshape(-1, 4, 4)
            if poses.shape[0] != n_views:
                raise ValueError(f"{n_views} views but {poses.shape[0]} poses")
            # uploaded once, before any compute-stream launch reads it
            poses = poses.to(self.eng.device).contiguous()
            torch.cuda.current_stream(self.eng.device).synchronize()
        free = queue.Queue()
        for k in range(self.slots):
            free.put(k)
        work: queue.Queue = queue.Queue()
        err: list = []
        px = self.H * self.W

        def d2h_worker():
            while True:
                item = work.get()
                if item is None:
                    return
                i, k, done = item
                try:
                    if err:
                        continue
                    with torch.cuda.stream(self._d2h):
                        self._d2h.wait_event(done)
                        cl = self._out[k]
                        self._hn[k][:2].copy_(cl["view_offsets"], non_blocking=True)
                        if self.count_masked:
                            self._hn[k][2:].copy_(self._mc[k], non_blocking=True)
                        self._d2h.synchronize()
                        if self.count_masked:
                            self._masked[i] = int(self._hn[k][2])
                        n = int(self._hn[k][1] - self._hn[k][0])
                        if on_device is not None:
                            on_device(i, cl["xyz"][:n], cl["bgr"][:n])
                        if consume is not None:
                            self._hx[k][:n].copy_(cl["xyz"][:n], non_blocking=True)
                            self._hb[k][:n].copy_(cl["bgr"][:n], non_blocking=True)
                            st.d2h_bytes += n * (3 * self._esz + 3)
                        self._d2h.synchronize()
                    st.points += n
                    st.per_view_points.append(n)
                    if consume is not None:
                        t0 = time.perf_counter()
                        consume(i, self._hx[k][:n].numpy(), self._hb[k][:n].numpy())
                        st.consume_s += time.perf_counter() - t0
                except BaseException as e:  # noqa: BLE001 -- re-raised on the caller's thread
                    err.append(e)
                finally:
                    free.put(k)

        th = threading.Thread(target=d2h_worker, name="sl-d2h", daemon=True)
        t_start = time.perf_counter()
        th.start()
        try:
            for i in range(n_views):
                k = free.get()
                if err:
                    break
                t0 = time.perf_counter()
                got = fill(i, self._hs[k], self._ht[k])
                st.fill_s += time.perf_counter() - t0
                if isinstance(got, HostView):
                    hs, ht = got.stack[: self.n_up], got.texture
                    if tuple(hs.shape) != (self.n_up, self.H, self.W) or hs.dtype != torch.uint8:
                        raise ValueError(f"HostView.stack must be uint8 [>={self.n_up},{self.H},{self.W}]")
                    if ht is not None and (tuple(ht.shape) != (self.H, self.W, 3) or ht.dtype != torch.uint8):
                        raise ValueError(f"HostView.texture must be uint8 [{self.H},{self.W},3]")
                else:
                    hs, ht = self._hs[k], (None if got else self._ht[k])
                gray_tex = ht is None
                with torch.cuda.stream(self._copy):
                    self._ds[k].copy_(hs, non_blocking=True)
                    if not gray_tex:
                        self._dt[k].copy_(ht, non_blocking=True)
                    up = torch.cuda.Event()
                    up.record(self._copy)
                st.h2d_bytes += hs.numel() + (0 if gray_tex else ht.numel())
                self._compute.wait_event(up)
                self.eng.decode_triangulate(self._ds[k], self.n_cols, self.n_rows,
                                            texture=None if gray_tex else self._dt[k], mask_mode=self.mask_mode,
                                            maps=False, cloud=True, xyz_dtype=self.xyz_dtype,
                                            poses=None if poses is None else poses[i], fast_f32=self.fast_f32,
                                            stream=self._compute, out=self._out[k],
                                            mask_counts=self._mc[k] if self.count_masked else None)
                done = torch.cuda.Event()
                done.record(self._compute)
                work.put((i, k, done))
                st.views += 1
                st.pixels += px
        finally:
            work.put(None)
            th.join()
        if err:
            raise err[0]
        self.eng.sync(self._compute)
        self._masked.clear()
        st.wall_s = time.perf_counter() - t_start
        return st
