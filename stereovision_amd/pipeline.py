"""Frames in flight for the host-buffer drop-in path.

The reference computes one frame pair per call and overlaps it with other work through a
worker pool (fused_depth_map.py:2299 creates a 2-worker ThreadPoolExecutor, :2591-2598
submits the stereo call, :2671 waits at most 0.5 s).  A synchronous call through one
context serialises its host staging copy, the PCIe transfers and the kernels.
:class:`DepthMapPipeline` keeps `depth` frames in flight on as many contexts of the same
device (own stream, pinned staging and device buffers each), one host thread per context,
so one frame's host copies overlap another's transfers and kernels.  Results are the same
arrays create_depth_map returns (depth_final, disparity, depth_colormap), bit-identical to
the synchronous call.
"""
from __future__ import annotations

import os
import queue
import threading
from concurrent.futures import Future

import numpy as np

from . import colormap
from .engine import Engine, get_engine


def max_in_flight() -> int:
    """Contexts (streams) worth keeping in flight on one device: two per hardware queue the HIP
    runtime maps one process's streams onto (GPU_MAX_HW_QUEUES, 4 by default and on the GPU
    boxes) — while one context's host work (page-locked staging, expansion of the medians into
    the output maps) runs, the other keeps the queue fed.  Measured at 1080p (profiles/
    r06_pipeline/sweep.txt, 40 warm-up frames and 3 x 300 timed per depth): depth 8 beats 4 by
    15-19 % in two sweeps; from 16 the per-call staging/issue time grows to 2.5-3 ms and the
    rate falls (24: 2.6k).  Round 5's "depth 6 loses to 4" was an artifact: that sweep warmed
    4 frames in all, so contexts 5 and 6 paid their first-use costs inside the timed region."""
    try:
        return 2 * max(1, int(os.environ.get("GPU_MAX_HW_QUEUES", "4")))
    except ValueError:
        return 8


class DepthMapPipeline:
    """submit(left, right) -> Future of create_depth_map's (depth_final, disparity,
    depth_colormap) on the MI355X engine, up to `depth` frames in flight."""

    def __init__(self, num_disp: int, window_size: int, min_disp: int = 0, min_depth: float = 0.3,
                 max_depth: float = 2.0, cost: str = "sad", depth: int = 3, device: int | None = None,
                 cmap: str = "turbo", cap: bool = True):
        """depth: frames in flight, capped at :func:`max_in_flight` (two contexts per hardware
        queue; deeper pipelines only add per-call staging time).  cap=False keeps the requested
        depth (for measuring the cap itself)."""
        self.num_disp, self.win, self.min_disp = int(num_disp), int(window_size), int(min_disp)
        self.min_depth, self.max_depth, self.cost = float(min_depth), float(max_depth), cost
        self.requested_depth = max(1, int(depth))
        self.depth = min(self.requested_depth, max_in_flight()) if cap else self.requested_depth
        first = get_engine(device)
        self._engines = [first] + [Engine(first.device) for _ in range(self.depth - 1)]
        self._own = self._engines[1:]
        self._table = colormap.table(cmap)
        self._q: queue.Queue = queue.Queue()
        self._threads = [threading.Thread(target=self._worker, args=(e,), daemon=True)
                         for e in self._engines]
        for t in self._threads:
            t.start()

    def _worker(self, eng: Engine):
        while True:
            item = self._q.get()
            if item is None:
                return
            fut, left, right = item
            if not fut.set_running_or_notify_cancel():
                continue
            try:
                fut.set_result(eng.depth_map_color(left, right, self.min_disp, self.num_disp, self.win,
                                                   self.min_depth, self.max_depth, self._table,
                                                   min_disp_global=self.min_disp, cost=self.cost))
            except BaseException as e:  # delivered through the future
                fut.set_exception(e)

    def submit(self, left: np.ndarray, right: np.ndarray) -> Future:
        fut: Future = Future()
        self._q.put((fut, left, right))
        return fut

    def close(self):
        for _ in self._threads:
            self._q.put(None)
        for t in self._threads:
            t.join()
        for e in self._own:
            e.close()
        self._own = []

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
